for i in 1 2; do
  for t in build_var/head .; do
    (cd $t && timeout -k 10 200 python3 bench.py --mode ae-train --cpu-seconds 0 > /tmp/ae.json 2>/dev/null; python3 -c "import json;d=json.load(open('/tmp/ae.json'));print('$t', round(d['value'],1), round(d['ms_per_step'],2), d.get('kernels_ms_per_step'))")
  done
done

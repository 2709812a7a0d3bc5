"""Alternating A/B runs of one bench mode under different environments (variant libraries through
AST_HIP_LIB, feature switches), each arm in a fresh process, ROUNDS rounds in interleaved order:
python scripts/ab_runs.py MODE ROUNDS "name:VAR=val,VAR2=val" ["name2:..." ...]
TREE=path (relative to the repo root) runs that arm's bench.py from another checkout (e.g. a git
worktree of the previous commit with its own in-tree libraries): A/B of Python and kernels together.
Prints per run: img/s, ms/step and the per-kernel-family ms/step of the bench line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    mode, rounds = sys.argv[1], int(sys.argv[2])
    arms = []
    for spec in sys.argv[3:]:
        name, _, env = spec.partition(":")
        kv = dict(e.split("=", 1) for e in env.replace(";", ",").split(",") if e)
        for k, v in kv.items():
            if k == "AST_HIP_LIB" and not os.path.isabs(v):
                kv[k] = os.path.join(ROOT, v)
        arms.append((name, kv))
    for rnd in range(rounds):
        for name, kv in (arms if rnd % 2 == 0 else arms[::-1]):
            env = dict(os.environ, **kv)
            tree = os.path.join(ROOT, env.pop("TREE")) if "TREE" in env else ROOT
            r = subprocess.run([sys.executable, os.path.join(tree, "bench.py"), "--mode", mode, "--cpu-seconds", "0",
                                "--steps", "10", "--warmup", "3"], env=env, cwd=tree, capture_output=True,
                               text=True, timeout=280)
            if r.returncode != 0:
                print(name, "FAILED", r.stderr[-1500:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            fam = {k: round(v["ms_per_step"], 2) for k, v in d.get("kernels", {}).items()}
            print(f"r{rnd} {name:10s} {d['value']:8.1f} img/s {d['ms_per_step']:8.2f} ms/step {fam}", flush=True)


if __name__ == "__main__":
    main()

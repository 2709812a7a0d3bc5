"""CPU oracle for the AdaIN hot path — TEST INFRASTRUCTURE ONLY (see ref_cpu.py header).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""

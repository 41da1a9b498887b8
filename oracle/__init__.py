"""oracle/ — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's hot path (BLS12-381 PS/Coconut verify, aggregate, PoK
verify).  Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg —
as the checker, never as the thing measured or shipped.
"""

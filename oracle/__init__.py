"""ORACLE — test infrastructure only (CPU restatements of the reference; see module headers).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only
as the checker or the timed CPU baseline. The product package never imports it.
"""

"""Test infrastructure: CPU oracle for the KFAC hot path (see kfac_oracle.py header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""

"""TEST INFRASTRUCTURE ONLY: Python handle on the C oracle (norm_fec_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""

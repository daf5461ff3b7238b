"""TEST INFRASTRUCTURE ONLY: CPU oracle of the SVO ray path (see svo_oracle.h).
Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""

"""CPU oracle (test infrastructure only; see lightgcn_oracle.py header)."""

"""CPU oracle — test infrastructure only (see cogvideox_oracle.py header)."""

"""Parity oracle — test infrastructure only (see nerf_oracle.py header)."""

"""Parity oracle (test infrastructure only -- never imported by the product path).

See nf_oracle.py for what it restates and how it is pinned to the reference.
"""

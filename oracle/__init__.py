"""CPU parity oracle (TEST INFRASTRUCTURE ONLY — see rt_oracle.h)."""

"""TEST INFRASTRUCTURE ONLY -- the CPU oracle (see oracle/dfq_oracle.c)."""

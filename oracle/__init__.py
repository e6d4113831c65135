"""CPU oracle package (test infrastructure only; see oracle/sdmm_oracle.h)."""

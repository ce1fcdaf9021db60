"""CPU oracle for the Merkle hot path -- TEST INFRASTRUCTURE ONLY (see merkle_oracle.c)."""

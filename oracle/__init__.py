"""CPU oracle package — TEST INFRASTRUCTURE ONLY (see ia_oracle.py header)."""

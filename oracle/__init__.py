"""CPU oracle for the HybridVAE path -- test infrastructure only (see ref_cpu.py)."""

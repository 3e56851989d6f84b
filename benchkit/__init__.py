"""Bench-side support of bench.py (not the product): the N>1 allreduce bench, its watchdog and
the reference benchmark's result table.  The product's Python face is hydra_amd/."""

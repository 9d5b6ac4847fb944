"""Device-side ops: the persistent HIP cycle engine (engine.py) and the CDNA4
micro-benchmark suite (ubench.py)."""

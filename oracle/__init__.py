"""ORACLE — test infrastructure only (CPU restatement used as the checker and as
bench.py's cpu_baseline).  Never imported by the product package."""

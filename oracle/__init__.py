"""ORACLE — test infrastructure only (see captioner.py header).  Never imported by the product."""

"""ORACLE — test infrastructure only (CPU restatement of the reference path)."""

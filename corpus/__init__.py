"""Synthetic corpus tooling for tests and bench (not part of the decode path)."""

"""Harness counterparts of the reference's scripts (same flags, same printouts)."""

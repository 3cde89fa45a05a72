"""Auxiliary command-line tools (reference tools/: csvdiff, csvconcatenate, tests.sh)."""

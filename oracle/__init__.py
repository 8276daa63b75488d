"""CPU oracle (test infrastructure only) -- see wfsa_oracle.c / oracle.py."""
from .oracle import ENUM, TRELLIS, Oracle, OracleError, build, lib  # noqa: F401

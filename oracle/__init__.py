"""CPU oracle for the EC + checksum hot path -- TEST INFRASTRUCTURE ONLY.

A restatement of the reference's Java algorithms (see ozec_oracle.c for file:line citations).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package; the
product path (ozone_amd/) never does.
"""
from .oracle import *  # noqa: F401,F403

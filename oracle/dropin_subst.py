#!/usr/bin/env python3
"""ORACLE TEST INFRASTRUCTURE (build container only): rewrite the
preprocessed reference src/streamer.f90 (stdin) so that its hot path goes
through the library's shim (oracle/harness/m_dropin.f90), stdout. Four
kinds of call change, nothing else: mg_init (its HYPRE set-up skipped),
every field_compute and field_from_potential, and the forward_euler handed
to af_advance for the densities.
The file itself never enters the repository (oracle/Makefile pipes it from
/root/reference into a temporary directory)."""
import sys

src = sys.stdin.read()
subs = [
    ("  use m_model\n", "  use m_model\n  use m_dropin\n", 1),
    ("time_integrator, forward_euler)", "time_integrator, dropin_forward_euler)", 1),
    ("call mg_init(tree, mg)", "call dropin_mg_init(tree, mg, cfg)", None),
    ("call field_compute(tree, mg,", "call dropin_field_compute(tree, mg,", None),
    ("call field_from_potential(tree, mg)", "call dropin_field_from_potential(tree, mg)", None),
]
for old, new, count in subs:
    n = src.count(old)
    if n == 0 or (count is not None and n != count):
        sys.exit("dropin_subst: %r found %d times" % (old, n))
    src = src.replace(old, new)
sys.stdout.write(src)

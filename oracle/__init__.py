"""CPU oracle for the DeepVCP registration hot path (REF-R semantics).

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline.  The
product path (``deepvcp-pointcloud-registration_amd/dvcp``) never imports it
and fails loudly when its HIP library is missing.

PARITY UNPINNED.  The reference repository ships no tests, golden vectors or
known-answer fixtures, and importing/running the
reference Python was denied in this pipeline.  The
oracle is therefore a line-by-line restatement of the reference's torch ops
(with the enumerated crash repairs R1-R7 of SURVEY.md Appendix A.2), pinned
only by hand-derived known-answer tests (``tests/test_oracle_kat.py``).
"""
from .ref_r import *  # noqa: F401,F403

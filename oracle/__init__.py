"""CPU oracle for the RE-GCN hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU and in plain PyTorch/numpy, the reference
algorithm of sgxxyyds/RE-GCN for the path named by BASELINE.json's north star
(per-timestep relational message passing + hyperbolic scoring).  Every function
cites the reference file:line it follows.  It mirrors the reference's op
sequence (per-edge message materialisation, per-edge GEMM for the Union layer,
per-destination Lorentz centroid, chunk-free all-pair scoring).

Who may use it: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — as the checker and the timed CPU baseline, never as the
thing measured or shipped.  The product package (re-gcn_amd/regcn_amd) never
imports this package and fails loudly without its HIP library.

Parity pinning: the oracle is pinned against golden vectors produced by
running the reference itself in the build container
(tools/goldens/make_golden.py -> tests/golden/*.npz, checked by
tests/test_oracle_golden.py).  DGL 0.5.2 (requirement.txt:3) is absent; its
message-passing semantics (builtin sum with zero fill, apply on all nodes,
degree-bucketed UDF reduce with zero fill) are restated by the test-only
stand-in in tools/goldens/standin, so the DGL boundary itself is unpinned
against real DGL.
"""

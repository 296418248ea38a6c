"""ORACLE — test infrastructure only.

CPU restatement of the reference's (Lolash/graphSAGE-pytorch) sample-and-
aggregate path, used exclusively as the checker by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg.  Nothing in the
product package imports it; the product path has no CPU fallback.

Parity pinning: the restatement is checked against golden vectors captured
from the reference itself in the build container (tests/golden/make_golden.py,
tests/test_oracle_golden.py): RNG known answers, set-order known answers,
per-hop frontiers/sampled sets, embeddings and weight gradients.
"""
from .reference_semantics import (  # noqa: F401
    Adjacency, sample_hop, sample_layers, forward_dense, train_step_dense, nll_loss,
)
from . import unsup_semantics  # noqa: F401

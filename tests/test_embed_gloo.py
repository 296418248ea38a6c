"""Rank sharding + all-gather of the multi-GPU get_gnn_embeddings (SURVEY
§8 f-3) on CPU, gloo, world size 2.  The per-rank native pipeline
(utils._embed_ids -> train.Embedder, GPU-only, covered by
tests/test_eval_utils.py) is replaced by a stand-in that tags every row with
its node id and the rank's stream count; the check is that every rank ends
with the [N, H] matrix in node order, each row computed exactly once, by the
rank that owns its batch (batch i on rank i % W)."""
import importlib
import os
import socket
import tempfile
import types

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

utils = importlib.import_module("graphsage-pytorch_amd.utils")

N, B, H, S = 23, 4, 5, 2


def _stand_in(calls):
    def embed(gnn_model, ids, b_sz, rngs):
        calls.append((ids.copy(), b_sz, len(rngs)))
        rank = dist.get_rank()
        base = torch.from_numpy(ids).double()[:, None] * torch.arange(1, H + 1, dtype=torch.float64)
        return (base + 1000.0 * rank).float()
    return embed


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    utils._embed_ids = _stand_in(calls)
    dc = types.SimpleNamespace(g_labels=np.zeros(N, np.int64))
    E = utils.get_gnn_embeddings(object(), dc, "g", b_sz=B, sampler_streams=S)
    torch.save(E, os.path.join(out_dir, f"E{rank}.pt"))
    np.save(os.path.join(out_dir, f"ids{rank}.npy"), calls[0][0])
    assert len(calls) == 1 and calls[0][1] == B and calls[0][2] == S
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_embeddings_all_gather_in_node_order():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        E = [torch.load(os.path.join(d, f"E{r}.pt"), weights_only=True) for r in range(world)]
        ids = [np.load(os.path.join(d, f"ids{r}.npy")) for r in range(world)]
    assert torch.equal(E[0], E[1])
    assert sorted(np.concatenate(ids).tolist()) == list(range(N))
    owner = (np.arange(N) // B) % world
    expect = torch.arange(N, dtype=torch.float64)[:, None] * torch.arange(1, H + 1, dtype=torch.float64)
    expect = (expect + 1000.0 * torch.from_numpy(owner).double()[:, None]).float()
    assert torch.equal(E[0], expect)

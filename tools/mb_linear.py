"""Microbenchmark of the SageLayer linear kernels at the rmat2m bench shapes.

Times each kernel with HIP events on torch's current stream, warm (back-to-back
repeats) and cold (a 512 MiB write between calls evicts L2/MALL), so kernel
latency can be separated from first-touch cost.  GPU only; not a test.
"""
import argparse
import importlib
import json
import sys

import torch

sys.path.insert(0, ".")
ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")


def timeit(fn, reps, cold, flush):
    evs = []
    for _ in range(reps):
        if cold:
            flush.fill_(1.0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--n1", type=int, default=4400)
    ap.add_argument("--n2", type=int, default=512)
    ap.add_argument("--F", type=int, default=256)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--nodes", type=int, default=1 << 21)
    ap.add_argument("--self-rows", choices=["random", "contiguous"], default="random",
                    help="layer-1 self rows: random rows of the 2M-row table, or a contiguous n-row block")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    F, H = args.F, args.H
    X = torch.rand(args.nodes, F, device=dev) - 0.5
    flush = torch.empty(128 << 20, device=dev)
    res = {}
    for name, n, fin, gather in (("layer1", args.n1, F, True), ("layer2", args.n2, H, False)):
        A = torch.rand(n, fin, device=dev) - 0.5
        Xs = X if gather else torch.rand(4 * n, fin, device=dev) - 0.5
        sidx = torch.randint(0, Xs.shape[0], (n,), device=dev, dtype=torch.int32)
        if gather and args.self_rows == "contiguous":
            Xs = X[:n].clone()
            sidx = torch.arange(n, device=dev, dtype=torch.int32)
        W = (torch.rand(H, 2 * fin, device=dev) - 0.5) * 0.1
        out = torch.empty(n, H, device=dev)
        dout = torch.randn(n, H, device=dev)
        dW = torch.empty(H, 2 * fin, device=dev)
        dIn = torch.empty(n, 2 * fin, device=dev)
        ws = ops.linear_dw_workspace(n, 2 * fin, H, dev)
        fns = {
            "fwd": lambda: ops.sage_linear_fwd(A, W, out, Xs=Xs, sidx=sidx, relu=True),
            "dw": lambda: ops.sage_linear_bwd_weight(A, dout, out, dW, Xs=Xs, sidx=sidx, relu=False, ws=ws),
            "dx": lambda: ops.sage_linear_bwd_input(dout, out, W, dIn[:, fin:], dSelf=dIn[:, :fin], relu=False),
        }
        ref = torch.relu(torch.cat([Xs[sidx.long()], A], 1) @ W.t())
        fns["fwd"]()
        torch.cuda.synchronize()
        err = (out - ref).abs().max().item()
        for k, fn in fns.items():
            warm = timeit(fn, args.reps, False, flush)
            cold = timeit(fn, max(10, args.reps // 5), True, flush)
            res[f"{name}.{k}"] = {"warm_us": round(warm, 2), "cold_us": round(cold, 2)}
        res[f"{name}.fwd"]["max_err"] = err
        flops = 2.0 * n * 2 * fin * H
        res[f"{name}.fwd"]["tflops_warm"] = round(flops / res[f"{name}.fwd"]["warm_us"] / 1e6, 2)
    tiny = torch.zeros(64, device=dev)
    res["tiny_add"] = {"warm_us": round(timeit(lambda: tiny.add_(1.0), args.reps, False, flush), 2),
                       "cold_us": round(timeit(lambda: tiny.add_(1.0), 10, True, flush), 2)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""One line per rocprof'd bench run for tools/ab_prof.sh: the rocprof average
(us) of each step kernel (its most-dispatched instance), the main-stream sum,
and the bench's steady / sustained ms per step; --summary: per-build medians."""
import collections
import glob
import json
import statistics
import sys

MAIN = ("linear_fwd_wide_kernel", "linear_dw_xcd_kernel", "sage_top_kernel", "layer_bwd_top_kernel",
        "sum_slabs_pair_kernel")
SIDE = ("agg_ids_kernel", "pull_pack_kernel", "resolve_top_kernel")
SHORT = {"linear_fwd_wide_kernel": "fwd", "linear_dw_xcd_kernel": "dw", "sage_top_kernel": "top",
         "layer_bwd_top_kernel": "bwdtop", "sum_slabs_pair_kernel": "slab", "agg_ids_kernel": "gather",
         "pull_pack_kernel": "pull", "resolve_top_kernel": "resolve"}


def line(name, d, log):
    import csv
    path = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))[0]
    best = {}
    for row in csv.DictReader(open(path)):
        for k in MAIN + SIDE:
            if k in row["Name"] and (k not in best or int(row["Calls"]) > best[k][0]):
                best[k] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    b = json.loads([x for x in open(log).read().splitlines() if x.startswith("{")][-1])
    main = sum(best[k][1] for k in MAIN if k in best)
    vals = " ".join(f"{SHORT[k]}={best[k][1]:.2f}" for k in MAIN + SIDE if k in best)
    print(f"{name} steady={1e3 * b['ms_per_step']:.1f} sustained={1e3 * b['sustained']['ms_per_step']:.1f} "
          f"main={main:.2f} {vals}")


def summary(path):
    r = collections.defaultdict(lambda: collections.defaultdict(list))
    for ln in open(path):
        f = ln.split()
        for kv in f[1:]:
            k, v = kv.split("=")
            r[f[0]][k].append(float(v))
    for so, d in r.items():
        print("median", so, " ".join(f"{k} {statistics.median(v):.2f}" for k, v in d.items()),
              " n", len(d["main"]))


if __name__ == "__main__":
    if sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        line(*sys.argv[1:4])

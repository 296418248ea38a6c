"""bench.py's lookups of the committed profiles (CPU): the rocprofv3 summary,
PMC traffic and MFMA busy of the layer-1 kernels are found under the names the
bench launches them with (parameter lists and the deferred-update flag of the
forward's template stripped)."""
import os

import bench


FWD = "void gs::linear_fwd_wide_kernel<float, 48, true, true, true>(int, int, int, int, float const*, long)"
DW = "void gs::linear_dw_xcd_kernel<float, true, false, true, true>(int, int, int)"


def test_kernel_key_drops_params_and_pending_flag():
    assert bench.kernel_key(FWD) == "void gs::linear_fwd_wide_kernel<float, 48, true, true>"
    assert bench.kernel_key(FWD.replace("true, true, true>", "true, true, false>")) == bench.kernel_key(FWD)
    assert bench.kernel_key(DW) == "void gs::linear_dw_xcd_kernel<float, true, false, true, true>"


def test_committed_profiles_resolve():
    for cfg in ("rmat2m", "rmat2m-max-bf16"):
        rel = bench.rocprof_stats_file(cfg, 512)
        assert rel is not None and os.path.exists(os.path.join(bench.ROOT, rel))
    tr = bench.load_traffic("rmat2m", 512, FWD)
    assert tr is not None and tr["hbm_bytes"] > 0
    for k in (FWD, DW):
        mb = bench.load_mfma_busy("rmat2m", k)
        assert mb is not None and 0.0 < mb["mfma_util"] < 1.0
    assert bench.load_mfma_busy("no-such-config", FWD) is None

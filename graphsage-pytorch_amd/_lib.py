"""ctypes binding of libgraphsage_amd.so (declared in include/graphsage_amd.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C graphsage-pytorch_amd/csrc``).  There is no fallback: if the library
is missing every entry point raises, so a GPU run can never silently execute
something other than the HIP kernels.

torch is imported before the library is loaded so that the HIP runtime torch
ships (SONAME libamdhip64.so.7) is the one the kernels bind to — one runtime,
one device context, torch's streams usable as ``hipStream_t``.
"""
import ctypes
import os

import torch  # noqa: F401  (must load first: shares its HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# GS_HOST_ASAN_LIB (sanitizer runs only, tools/asan_host_tests.sh): load the
# host-only ASan/UBSan build of the library (host/*.cpp, no HIP) instead; the
# device entry points are then absent and raise if called.
_ASAN_LIB = os.environ.get("GS_HOST_ASAN_LIB")
LIB_PATH = _ASAN_LIB or os.path.join(_HERE, "libgraphsage_amd.so")

GS_OK, GS_EINVAL, GS_ENOMEM, GS_EHIP, GS_ERANGE, GS_EEMPTY, GS_ELIMIT = range(7)
GS_F32, GS_BF16 = 0, 1
GS_AGG_MEAN, GS_AGG_MAX = 0, 1
GS_SAMPLE_GCN, GS_SAMPLE_FULL = 1, 2
GS_DSAMPLER_NO_AUX = 8  # gs_dsampler_create: every kernel on the caller's stream
GS_MAX_HOPS = 8
GS_TOPT_FUSED_BWD, GS_TOPT_TOP_LAUNCH, GS_TOPT_SELF_ROWS, GS_TOPT_DEFER_UPDATE, GS_TOPT_TOP_PAIR = range(5)
(GS_PK_POS_PTR, GS_PK_POS, GS_PK_DST_IDS, GS_PK_NBR_PTR, GS_PK_NBR, GS_PK_SELF,
 GS_PK_TPTR, GS_PK_TIDX, GS_PK_NFIELDS) = range(9)

_i32, _i64, _u32, _u64, _f32, _f64 = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                      ctypes.c_uint64, ctypes.c_float, ctypes.c_double)
_vp = ctypes.c_void_p
_p = ctypes.POINTER


class HopView(ctypes.Structure):
    _fields_ = [
        ("n_dst", _i64), ("n_pos", _i64), ("n_src", _i64), ("n_nbr", _i64),
        ("dst_ids", _p(_i64)), ("pos_ptr", _p(_i32)), ("pos", _p(_i32)),
        ("src_ids", _p(_i64)), ("nbr_ptr", _p(_i32)), ("nbr", _p(_i32)),
        ("self_local", _p(_i32)), ("set_ptr", _p(_i32)), ("set_items", _p(_i64)),
        ("n_empty", _i64),
    ]


class PackLayout(ctypes.Structure):
    _fields_ = [("total", _i64), ("off", (_i64 * GS_PK_NFIELDS) * GS_MAX_HOPS)]


# name -> (restype, argtypes)
_SIGS = {
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_version": (ctypes.c_char_p, []),
    "gs_rng_create": (_i32, [_p(_vp)]),
    "gs_rng_destroy": (None, [_vp]),
    "gs_rng_seed_words": (_i32, [_vp, _vp, _i64]),
    "gs_rng_set_state": (_i32, [_vp, _vp, _i64]),
    "gs_rng_get_state": (_i32, [_vp, _vp, _p(_i64)]),
    "gs_rng_getrandbits": (_i32, [_vp, _i32, _i64, _vp]),
    "gs_rng_randbelow": (_i32, [_vp, _u32, _i64, _vp]),
    "gs_rng_sample_positions": (_i32, [_vp, _i64, _i64, _vp]),
    "gs_rng_choice_position": (_i32, [_vp, _i64, _p(_i64)]),
    "gs_pyset_union_of_lists": (_i32, [_vp, _vp, _i64, _vp, _p(_i64)]),
    "gs_graph_build": (_i32, [_vp, _vp, _i64, _i64, _i32, _p(_vp)]),
    "gs_graph_from_tables": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _p(_vp)]),
    "gs_graph_destroy": (None, [_vp]),
    "gs_graph_dims": (_i32, [_vp, _p(_i64), _p(_i64), _p(_i64)]),
    "gs_graph_row_ptr": (_vp, [_vp]),
    "gs_graph_col": (_vp, [_vp]),
    "gs_graph_image_bytes": (_i64, [_vp]),
    "gs_graph_write_image": (_i32, [_vp, _vp, _i64]),
    "gs_graph_from_image": (_i32, [_vp, _i64, _p(_vp)]),
    "gs_rmat_pairs": (_i32, [_i32, _i64, _f64, _f64, _f64, _u64, _i32, _i32, _vp, _vp, _p(_i64)]),
    "gs_sample_run": (_i32, [_vp, _vp, _vp, _i64, _vp, _i32, _i32, _p(_vp)]),
    "gs_sample_destroy": (None, [_vp]),
    "gs_sample_n_hops": (_i32, [_vp, _p(_i32)]),
    "gs_sample_hop": (_i32, [_vp, _i32, _p(HopView)]),
    "gs_sample_pack_layout": (_i32, [_vp, _p(PackLayout)]),
    "gs_sample_pack": (_i32, [_vp, _vp, _i64]),
    "gs_sample_pack_bound": (_i64, [_vp, _i64, _vp, _i32]),
    "gs_sample_pack_run": (_i32, [_vp, _vp, _vp, _i64, _vp, _i32, _i32, _vp, _i64, _vp, _vp, _p(_i64)]),
    "gs_sample_pack_bound_multi": (_i64, [_vp, _i64, _i64, _vp, _i32]),
    "gs_sample_pack_run_multi": (_i32, [_vp, _vp, _vp, _i64, _i64, _vp, _i32, _i32, _vp, _i64, _vp, _vp,
                                        _p(_i64)]),
    "gs_team_create": (_i32, [_i32, _p(_vp)]),
    "gs_team_create_shared": (_i32, [_vp, _p(_vp)]),
    "gs_team_destroy": (None, [_vp]),
    "gs_sample_pack_run_multi_team": (_i32, [_vp, _vp, _vp, _i64, _i64, _vp, _i32, _i32, _vp, _i64, _vp,
                                             _vp, _p(_i64), _vp]),
    "gs_fill_uniform": (_i32, [_vp, _i32, _i64, _i64, _i64, _u64, _vp]),
    "gs_uniform_host": (_i32, [_u64, _i64, _i64, _i64, _vp]),
    "gs_agg_fwd": (_i32, [_i32, _i32, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i32,
                          _vp, _i32, _i64, _vp, _vp]),
    "gs_sage_linear_fwd": (_i32, [_i32, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp,
                                  _i64, _i32, _vp]),
    "gs_sage_linear_bwd_weight_ws": (_i64, [_i64, _i64, _i64]),
    "gs_sage_linear_bwd_weight": (_i32, [_i32, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp,
                                         _vp, _i64, _i32, _vp, _vp, _i64, _vp]),
    "gs_sage_linear_bwd_input": (_i32, [_i64, _i64, _i64, _vp, _vp, _i64, _i32, _vp, _vp, _vp,
                                        _i64, _vp]),
    "gs_agg_bwd": (_i32, [_i32, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp,
                          _vp]),
    "gs_sage1_fwd_supported": (_i32, [_i32, _i64, _i64, _i32]),
    "gs_sage1_fwd": (_i32, [_i32, _i32, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i32,
                            _vp, _vp, _i64, _vp, _i64, _i32, _vp]),
    "gs_cls_nll_ws_floats": (_i64, [_i64, _i64, _i64]),
    "gs_cls_nll_fwd_bwd": (_i32, [_i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp,
                                  _vp, _vp, _vp]),
    "gs_clip_sgd": (_i32, [_i32, _vp, _vp, _vp, _f32, _f32, _f32, _vp, _vp]),
    "gs_unsup_create": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _p(_vp)]),
    "gs_unsup_destroy": (None, [_vp]),
    "gs_unsup_attach_device": (_i32, [_vp, _vp]),
    "gs_unsup_extend": (_i32, [_vp, _vp, _vp, _i64, _i64, _i32, _i32, _vp]),
    "gs_unsup_fetch": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gs_unsup_loss_plan": (_i32, [_vp, _vp, _i64, _vp, _p(_i64)]),
    "gs_unsup_loss_ws_floats": (_i64, [_i64, _i64, _i64]),
    "gs_unsup_loss_fwd": (_i32, [_i32, _i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _f32, _f32, _vp, _vp,
                                 _vp]),
    "gs_unsup_loss_bwd": (_i32, [_i64, _i64, _i64, _i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gs_cast_f32_bf16": (_i32, [_vp, _vp, _i64, _vp]),
    "gs_trainer_create": (_i32, [_vp, _p(_vp)]),
    "gs_trainer_destroy": (None, [_vp]),
    "gs_trainer_n_params": (_i64, [_vp]),
    "gs_trainer_ws_bytes": (_i64, [_vp, _vp]),
    "gs_trainer_forward_backward": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp]),
    "gs_trainer_update": (_i32, [_vp, _f32, _vp, _vp]),
    "gs_trainer_update_local": (_i32, [_vp, _vp]),
    "gs_trainer_defer": (_i32, [_vp, _i32, _p(_i32), _vp]),
    "gs_trainer_gather_reserve": (_i32, [_vp, _i64, _i32]),
    "gs_trainer_gather": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp]),
    "gs_trainer_forward_backward_gathered": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    "gs_trainer_forward": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "gs_trainer_forward_gathered": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp]),
    "gs_trainer_time_agg": (_i32, [_vp, _i64]),
    "gs_trainer_agg_times": (_i64, [_vp, _vp, _i64]),
    "gs_trainer_kernel_times": (_i64, [_vp, _i32, _vp, _i64]),
    "gs_trainer_kernel_block_stats": (_i64, [_vp, _i32, _vp, _i64]),
    "gs_trainer_kernel_stamps": (_i64, [_vp, _i32, _i64, _vp, _vp]),
    "gs_trainer_time_kernels": (_i32, [_vp, _i32, _i64]),
    "gs_trainer_time_kernels_every": (_i32, [_vp, _i32, _i64, _i64]),
    "gs_trainer_kernel_name": (ctypes.c_char_p, [_vp, _i32]),
    "gs_trainer_grads": (_vp, [_vp]),
    "gs_trainer_set_option": (_i32, [_vp, _i32, _i32]),
    "gs_trainer_capture": (_i32, [_vp, _vp, _i64, _vp, _i64]),
    "gs_trainer_captured": (_i64, [_vp]),
    "gs_comm_unique_id": (_i32, [_vp]),
    "gs_comm_create": (_i32, [_vp, _i32, _i32, _p(_vp)]),
    "gs_comm_destroy": (None, [_vp]),
    "gs_comm_allreduce_sum": (_i32, [_vp, _vp, _i64, _vp]),
    "gs_runner_create": (_i32, [_vp, _p(_vp)]),
    "gs_runner_run": (_i32, [_vp, _i64, _vp, _vp]),
    "gs_runner_stats_get": (_i32, [_vp, _vp]),
    "gs_runner_stats_reset": (None, [_vp]),
    "gs_runner_destroy": (None, [_vp]),
    "gs_runner_release": (_i32, [_vp, _i64]),
    "gs_runner_progress": (_i32, [_vp, _p(_i64), _p(_i64)]),
    "gs_runner_sync_rngs": (_i32, [_vp]),
    "gs_dsampler_create": (_i32, [_vp, _vp, _i32, _i64, _i32, _p(_vp)]),
    "gs_dsampler_destroy": (None, [_vp]),
    "gs_dsampler_set_rng": (_i32, [_vp, _vp, _i64, _vp]),
    "gs_dsampler_get_rng": (_i32, [_vp, _vp, _p(_i64), _vp]),
    "gs_dsampler_words": (_i32, [_vp, _i64, _vp, _vp]),
    "gs_dsampler_pack_bound": (_i64, [_vp, _i64]),
    "gs_dsampler_run": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp]),
    "gs_dsampler_result": (_i32, [_vp, _vp, _vp, _p(_i64)]),
    "gs_dsampler_runs": (_i64, [_vp]),
    "gs_dsampler_result_of": (_i32, [_vp, _i64, _vp, _vp, _p(_i64)]),
    "gs_dsampler_debug": (_i32, [_vp, _vp, _i32]),
}


class TrainerConfig(ctypes.Structure):
    _fields_ = [
        ("n_layers", _i32), ("hidden", _i32), ("n_classes", _i32), ("agg", _i32), ("gcn", _i32),
        ("feat_dtype", _i32), ("feat_dim", _i64), ("feat_ld", _i64),
        ("X", _vp), ("row_ptr", _vp), ("col", _vp), ("labels", _vp), ("params", _vp), ("grads", _vp),
        ("lr", _f32), ("max_norm", _f32),
    ]


class RunnerConfig(ctypes.Structure):
    _fields_ = [
        ("graph", _vp), ("trainer", _vp), ("batches", _vp), ("n_batches", _i64), ("batch", _i64),
        ("fanouts", _vp), ("n_hops", _i32), ("flags", _i32), ("n_streams", _i32), ("rngs", _vp),
        ("depth", _i32), ("comm", _vp), ("world", _i32), ("embed_out", _vp), ("embed_ld", _i64),
        ("merge", _i32), ("hold", _i32), ("ar_buckets", _i32), ("helpers", _i32), ("warm", _i32),
        ("device_sampler", _i32),
    ]


class RunnerStats(ctypes.Structure):
    _fields_ = [
        ("steps", _i64), ("wait_s", ctypes.c_double), ("issue_s", ctypes.c_double),
        ("sample_s", ctypes.c_double), ("hop_sizes", ctypes.c_double * (4 * GS_MAX_HOPS)),
        ("wait_sample_s", ctypes.c_double), ("wait_ring_s", ctypes.c_double),
        ("wait_gather_s", ctypes.c_double), ("fwd_bwd_s", ctypes.c_double), ("update_s", ctypes.c_double),
        ("max_step_s", ctypes.c_double), ("lookahead_misses", _i64),
    ]


_lib = None


class LibraryMissing(RuntimeError):
    pass


class DeviceLimit(RuntimeError):
    """GS_ELIMIT: a device-path capacity (the device sampler's rejection
    windows, walks or frontier tables) was too small for this batch.  The
    batch itself is valid and the caller's stream state is untouched, so the
    host path computes the same result."""


# measurement-only entry points a bench run may do without (an A/B against a
# library built before them); everything else must be exported
_DIAGNOSTIC = {"gs_trainer_kernel_block_stats", "gs_trainer_kernel_stamps"}


def lib():
    """Load (once) and return the configured ctypes library."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} is not built; run __graft_entry__.build() or "
                "`make -C graphsage-pytorch_amd/csrc` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)  # CDLL releases the GIL around every call
        for name, (res, args) in _SIGS.items():
            if (_ASAN_LIB or name in _DIAGNOSTIC) and not hasattr(L, name):
                continue  # device entry point: not in the host-only sanitizer build
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, what=""):
    """Raise the reference's exception type for a non-zero status."""
    if rc == GS_OK:
        return
    msg = lib().gs_last_error().decode(errors="replace") or what
    if rc in (GS_EINVAL,):
        raise ValueError(msg)
    if rc == GS_ERANGE:
        # random.sample: ValueError; unknown node ids: IndexError (features[node])
        raise (ValueError if "Sample larger" in msg else IndexError)(msg)
    if rc == GS_EEMPTY:
        raise IndexError(msg)
    if rc == GS_ENOMEM:
        raise MemoryError(msg)
    if rc == GS_ELIMIT:
        raise DeviceLimit(msg)
    raise RuntimeError(msg)


def ptr(t):
    """Raw address of a torch tensor / numpy array (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return t.ctypes.data


def stream_ptr(device=None):
    """hipStream_t of torch's current stream on `device`."""
    return torch.cuda.current_stream(device).cuda_stream

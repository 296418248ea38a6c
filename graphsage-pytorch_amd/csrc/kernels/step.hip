// Native training-step runtime: the reference's per-batch loop body
// (utils.py:157-191 — GraphSage forward, Classification + NLL, backward,
// clip_grad_norm_ per model, SGD) issued as one stream of the kernels in this
// library, with every intermediate carved from one caller-owned workspace.
// The Python host makes two calls per step (forward_backward, update) and
// puts the RCCL gradient all-reduce between them.
#include <cxxabi.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "internal.hpp"

struct gs_trainer {
    gs_trainer_config cfg;
    std::vector<int64_t> w_off;  // element offset of each parameter in the flat buffer
    std::vector<int64_t> w_rows, w_cols;
    int64_t cls_w_off = 0, cls_b_off = 0, total = 0;
    // optional kernel-bound HIP-event timing (bench roofline): site 0 the
    // layer-1 gather-aggregate, 1 the layer-1 linear forward, 2 its weight
    // gradient (the MFMA kernels), 3 the fused top layer + loss head (top.hip),
    // 4 the step's slab-sum pair launch (sum_slabs_pair_launch)
    static constexpr int kSites = 5;
    struct Timer {
        std::vector<hipEvent_t> ev0, ev1;
        int64_t n = 0;
        int64_t every = 1, calls = 0;  // time one launch of every `every`, the last of each run
        std::string kernel;  // demangled name of the kernel the site last timed
        // sites 1-4: the kernel's own span (KStamp, kcommon.hpp) per entry,
        // when the launch took it (else the entry's events timed it)
        unsigned long long* st0 = nullptr;  // device: per entry, kStampBlocks workgroup starts (100 MHz ticks)
        unsigned long long* st1 = nullptr;  // device: per entry, the workgroup ends
        std::vector<char> stamped;
    } timer[kSites];
    std::vector<hipEvent_t>& ev0 = timer[0].ev0;
    std::vector<hipEvent_t>& ev1 = timer[0].ev1;
    int64_t& n_timed = timer[0].n;
    // layer-1 aggregate slots for gathers issued ahead of their step
    // (gs_trainer_gather), so the next batch's gather overlaps this backward
    static constexpr int kSlots = 3;
    void* a1_slot[kSlots] = {};
    int64_t a1_rows = 0;
    // Each gather slot is [self | agg] rows of 2F (option GS_TOPT_SELF_ROWS,
    // default on; applied at gs_trainer_gather_reserve): the side-stream gather
    // also copies the layer-1 rows' own features, so the layer-1 forward and dW
    // read one dense block (no self-index round).  self_in_slot: the slot's self
    // half was written.
    bool self_rows = false;
    bool self_in_slot[kSlots] = {};
    // per slot, the layer-1 neighbour ids resolved ahead of the gather
    // (k_ids slots per destination), when reserved with a fanout
    int32_t* ids_slot[kSlots] = {};
    int k_ids = 0;
    // padded hop-1 records for the fused top launch, per gather slot (trainer_reserve_top)
    int32_t* top_slot[kSlots] = {};
    bool top_ready[kSlots] = {};
    int64_t top_rows = 0;
    int top_k = 0;
    // per gather slot, the layer-2 backward's records of the transposed hop-1
    // lists (8 ints per layer-1 row, rec_rows rows; written with the top records)
    int32_t* rec_slot[kSlots] = {};
    int64_t rec_rows = 0;
    bool rec_ready[kSlots] = {};
    // clip-norm partials produced by the fused backward's reduce launches
    // (group 0: the sage weights' slab sums, group 1: the classifier reduce),
    // consumed by gs_trainer_update_local when no all-reduce came between
    // gs_trainer_set_option switches (alternatives the tests compare with the
    // default: bitwise, except top_launch, which matches within fp32 rounding)
    bool fuse_bwd = true;    // GS_TOPT_FUSED_BWD: layers >= 2 backward in fused launches
    bool use_top = true;     // GS_TOPT_TOP_LAUNCH: layer 2 + loss head + dIn2 in one launch
    bool want_self_rows = true;  // GS_TOPT_SELF_ROWS
    bool opt_defer = true;   // GS_TOPT_DEFER_UPDATE: runner loops defer each clip + SGD
    bool opt_top_pair = false;  // GS_TOPT_TOP_PAIR: the top launch on two blocks per 4 roots (C <= 16);
                                // off: measured neutral in the step (DESIGN.md §4 top)
    // the pair form's exchange: tagged granules ([quads][2][64], zeroed when
    // allocated), this trainer's launch tag and the give-up flag
    unsigned long long* xch = nullptr;
    int64_t xch_quads = 0;  // (words of xch)
    unsigned xch_epoch = 0;
    unsigned* xch_fail = nullptr;
    float* norm_part = nullptr;
    int pstride = 0;
    int npart[2] = {0, 0};
    bool norm_ready = false;
    std::function<void(hipStream_t)> upper_hook;  // internal.hpp trainer_set_upper_hook
    std::function<void(hipStream_t, int64_t, int64_t)> w1_chunk_hook;  // trainer_set_w1_chunk_hook
    int w1_chunks = 1;
    // bf16 features: W1 in bf16 for the layer-1 forward.  Cast from the fp32
    // W1 before a forward, except inside a runner loop (lp_keep), where the
    // SGD launch writes it beside W1 (g_lowp_shadow) and it stays valid from
    // one step to the next: nothing else writes the parameters there.
    uint16_t* w1_lp = nullptr;
    bool lp_keep = false, lp_valid = false;
    // Deferred update (trainer_defer_update, runner loops without an
    // all-reduce): a step's clip + SGD is not a launch of its own.  The step's
    // last slab sum writes W1's update for clip coefficient 1 into the other
    // W1 buffer, and the next step's layer-1 forward applies the pending
    // update (FwdSpec, kcommon.hpp): W1 from that buffer (or recomputed there
    // when the coefficient is not 1), the other parameters in its prologue.
    // The current W1 lives in w1_buf(w1_cur): buffer 0 is its place in the
    // flat params, buffer 1 w1_alt; trainer_defer_update(false) puts the
    // result of the last pending update back into the flat params.
    bool defer = false, pending = false;
    bool defer_comm = false;  // the all-reduce path: gs_trainer_update leaves the update pending
    // the pending update's norm partials (the step's own, or gs_trainer_update's
    // after the all-reduce), per-group counts and stride, gradient scale
    const float* pend_part = nullptr;
    int pend_pstride = 0;
    int pend_np[2] = {0, 0};
    float pend_scale = 1.f;
    float* w1_alt = nullptr;
    int w1_cur = 0;
    float* w1_buf(int i) { return i == 0 ? cfg.params + w_off[0] : w1_alt; }
    // bf16 features: the forward's bf16 W1 beside each buffer (lp_buf(w1_cur)
    // is current while deferring: the slab sum and the recompute write both)
    uint16_t* w1_lp_alt = nullptr;
    uint16_t* lp_buf(int i) { return i == 0 ? w1_lp : w1_lp_alt; }
    // Parity capture (gs_trainer_capture; tests only): after each training
    // step's launches, the step's root embeddings (the top layer's output) and
    // the flat gradient as the step left it (before its clip + SGD) are copied
    // on the step's stream into caller buffers.
    struct Capture {
        float* emb = nullptr;
        int64_t emb_stride = 0;
        float* grads = nullptr;
        int64_t max_steps = 0, n = 0;
    } cap;
    const float* last_emb = nullptr;  // the last run_step's [B, H] top-layer output
    ~gs_trainer() {
        if (w1_alt) (void)hipFree(w1_alt);
        if (w1_lp_alt) (void)hipFree(w1_lp_alt);
        if (norm_part) (void)hipFree(norm_part);
        if (xch) (void)hipFree(xch);
        if (xch_fail) (void)hipFree(xch_fail);
        if (w1_lp) (void)hipFree(w1_lp);
        for (auto& tm : timer) {
            for (auto e : tm.ev0) (void)hipEventDestroy(e);
            for (auto e : tm.ev1) (void)hipEventDestroy(e);
        }
        for (void* p : a1_slot)
            if (p) (void)hipFree(p);
        for (int32_t* p : ids_slot)
            if (p) (void)hipFree(p);
        for (int32_t* p : top_slot)
            if (p) (void)hipFree(p);
        for (int32_t* p : rec_slot)
            if (p) (void)hipFree(p);
        for (auto& tm : timer)
            if (tm.st0) (void)hipFree(tm.st0);
    }
};

namespace gs {

// Bump allocator over the workspace (256-byte aligned carves).
struct Carve {
    char* base;
    int64_t cap, at = 0;
    template <class T>
    T* take(int64_t n) {
        at = (at + 255) & ~int64_t(255);
        T* p = base ? reinterpret_cast<T*>(base + at) : nullptr;
        at += n * static_cast<int64_t>(sizeof(T));
        return p;
    }
};

struct HopSz {
    int64_t n_dst, n_pos, n_src, n_nbr;
};

static inline void ok(int rc) {
    if (rc != GS_OK) fail(rc, gs_last_error());
}

// Bind the next launch_k launch to timer site `site` when it has capacity
// left; returns whether it did (pass the result to timed_done).
static inline bool timed_arm(gs_trainer& T, int site) {
    auto& tm = T.timer[site];
    if (tm.n >= static_cast<int64_t>(tm.ev0.size())) return false;
    if (++tm.calls % tm.every) return false;
    g_launch_events = {tm.ev0[tm.n], tm.ev1[tm.n]};
    if (tm.st0) g_kernel_stamp = {tm.st0 + tm.n * kStampBlocks, tm.st1 + tm.n * kStampBlocks};
    g_launch_name = nullptr;  // set by the timed launch
    return true;
}
// Timer events only measure: no system-scope release when they complete (a
// system-scope release writes back and invalidates the caches under the work
// that follows, which is what made event-bound launches cost the step time).
static unsigned timer_event_flags() { return hipEventDisableSystemFence; }

static std::string demangle(const char* sym) {
    if (!sym) return "?";
    int status = 0;
    char* d = abi::__cxa_demangle(sym, nullptr, nullptr, &status);
    std::string out = (status == 0 && d) ? d : sym;
    std::free(d);
    return out;
}

static inline void timed_done(gs_trainer& T, int site, bool armed) {
    if (!armed) return;
    auto& tm = T.timer[site];
    if (tm.st0) tm.stamped[tm.n] = g_kernel_stamp.start == nullptr;  // the launch took the stamp
    g_kernel_stamp = {};
    GS_REQUIRE(!g_launch_events.start, GS_EINVAL, "timed launch did not consume its events");
    // the kernel of the latest timed launch (the layer-1 forward has two instances:
    // with the deferred update pending, and without, at a run's first step)
    if (g_launch_name) T.timer[site].kernel = demangle(g_launch_name);
    ++T.timer[site].n;
}

// The layer-1 gather-aggregate of one packed sample (models.py:291-330 at
// layer 1) into `out`, bracketed by the timing events when armed.
static void gather1(gs_trainer& T, const int32_t* pack, const int64_t* hop_sizes, const int64_t* offsets,
                    void* out, hipStream_t st, int64_t ldo = 0) {
    const gs_trainer_config& c = T.cfg;
    const int L = c.n_layers;
    const int64_t F = c.feat_dim;
    auto fld = [&](int f) -> const int32_t* {
        const int64_t o = offsets[(L - 1) * GS_PK_NFIELDS + f];
        GS_REQUIRE(o >= 0, GS_EINVAL, "pack field missing");
        return pack + o;
    };
    const bool timed = timed_arm(T, 0);
    ok(gs_agg_fwd(static_cast<gs_agg>(c.agg), static_cast<gs_dtype>(c.feat_dtype), c.X, c.feat_ld, F,
                  hop_sizes[4 * (L - 1)], fld(GS_PK_POS_PTR), fld(GS_PK_POS), nullptr, c.col, fld(GS_PK_DST_IDS),
                  c.gcn, out, static_cast<gs_dtype>(c.feat_dtype), ldo > 0 ? ldo : F, nullptr, st));
    timed_done(T, 0, timed);
}

// The same aggregate in two launches on `st`: resolve the sampled positions
// into padded neighbour ids, then gather rows through them (the timed launch;
// bitwise the expand-mode result).
static void gather1_ids(gs_trainer& T, const int32_t* pack, const int64_t* hop_sizes, const int64_t* offsets,
                        int slot, hipStream_t st) {
    const gs_trainer_config& c = T.cfg;
    const int L = c.n_layers;
    auto fld = [&](int f) -> const int32_t* {
        const int64_t o = offsets[(L - 1) * GS_PK_NFIELDS + f];
        GS_REQUIRE(o >= 0, GS_EINVAL, "pack field missing");
        return pack + o;
    };
    const int64_t n_dst = hop_sizes[4 * (L - 1)];
    int32_t* ids = T.ids_slot[slot];
    const int64_t n_top = hop_sizes[0];
    T.top_ready[slot] = T.top_k > 0 && L == 2 && !c.gcn && n_top <= T.top_rows && T.top_slot[slot] &&
                        hop_sizes[3] <= n_top * T.top_k;  // every root's list fits tk slots
    const int64_t n_rec = hop_sizes[2];  // |L1|: hop 1's sources
    T.rec_ready[slot] = T.top_ready[slot] && T.rec_slot[slot] && n_rec <= T.rec_rows;
    if (T.top_ready[slot]) {
        auto f1 = [&](int f) -> const int32_t* {
            const int64_t o = offsets[f];  // hop 1
            GS_REQUIRE(o >= 0, GS_EINVAL, "pack field missing");
            return pack + o;
        };
        resolve_top_launch(n_dst, T.k_ids, fld(GS_PK_POS_PTR), fld(GS_PK_POS), c.col, fld(GS_PK_DST_IDS), c.gcn, ids,
                           n_top, T.top_k, f1(GS_PK_NBR_PTR), f1(GS_PK_NBR), f1(GS_PK_SELF), T.top_slot[slot], st,
                           T.rec_ready[slot] ? n_rec : 0, f1(GS_PK_TPTR), f1(GS_PK_TIDX), T.rec_slot[slot]);
    } else {
        resolve_ids_launch(n_dst, T.k_ids, fld(GS_PK_POS_PTR), fld(GS_PK_POS), c.col, fld(GS_PK_DST_IDS), c.gcn, ids,
                           st);
    }
    const bool timed = timed_arm(T, 0);
    if (T.self_rows) {  // [self | agg] rows
        char* base = static_cast<char*>(T.a1_slot[slot]);
        const int64_t xsz = c.feat_dtype == GS_BF16 ? 2 : 4;
        agg_ids_launch(static_cast<gs_agg>(c.agg), static_cast<gs_dtype>(c.feat_dtype), c.X, c.feat_ld, c.feat_dim,
                       n_dst, T.k_ids, ids, fld(GS_PK_DST_IDS), c.gcn, base + c.feat_dim * xsz, 2 * c.feat_dim, st,
                       base, 2 * c.feat_dim);
        T.self_in_slot[slot] = true;
    } else {
        agg_ids_launch(static_cast<gs_agg>(c.agg), static_cast<gs_dtype>(c.feat_dtype), c.X, c.feat_ld, c.feat_dim,
                       n_dst, T.k_ids, ids, fld(GS_PK_DST_IDS), c.gcn, T.a1_slot[slot], c.feat_dim, st);
    }
    timed_done(T, 0, timed);
}

// Runs (or, with ws == nullptr, only sizes) one forward + backward.  With
// a1_slot >= 0 the layer-1 aggregate was produced by gs_trainer_gather.  With
// embed_out the step is the forward alone (models.py:241-269 as called by
// get_gnn_embeddings, utils.py:59-78): the last layer writes its [B, H]
// embeddings straight into embed_out and nothing after the forward runs.
static void top_pair_reserve(gs_trainer& t, int64_t B, hipStream_t st);

int64_t run_step(gs_trainer& T, const int32_t* pack, const int64_t* hop_sizes, const int64_t* offsets,
                        const int32_t* roots, int64_t B, char* ws, int64_t ws_bytes, float* loss,
                        hipStream_t st, int a1_slot = -1, float* embed_out = nullptr) {
    const gs_trainer_config& c = T.cfg;
    const int L = c.n_layers;
    const int64_t H = c.hidden, F = c.feat_dim;
    const bool lowp = c.feat_dtype == GS_BF16;
    const size_t xsz = lowp ? 2 : 4;
    std::vector<HopSz> hs(L);
    for (int j = 0; j < L; ++j) hs[j] = {hop_sizes[4 * j], hop_sizes[4 * j + 1], hop_sizes[4 * j + 2], hop_sizes[4 * j + 3]};
    auto fld = [&](int hop, int f) -> const int32_t* {  // hop 1-based
        const int64_t o = offsets[(hop - 1) * GS_PK_NFIELDS + f];
        GS_REQUIRE(o >= 0, GS_EINVAL, "pack field missing");
        return pack + o;
    };
    GS_REQUIRE(hs[0].n_dst == B, GS_EINVAL, "roots / hop-1 size mismatch");
    Carve cv{ws, ws_bytes};
    // ---- activations
    std::vector<void*> agg(L);
    std::vector<float*> h(L);
    std::vector<int32_t*> am(L, nullptr);
    std::vector<int64_t> rows(L), in_dim(L);
    for (int l = 1; l <= L; ++l) {
        const int j = L - l + 1;
        rows[l - 1] = hs[j - 1].n_dst;
        in_dim[l - 1] = l == 1 ? F : H;
        if (l == 1) {
            if (a1_slot >= 0) {
                GS_REQUIRE(rows[0] <= T.a1_rows && T.a1_slot[a1_slot], GS_EINVAL, "gather slot too small");
                agg[0] = T.a1_slot[a1_slot];
            } else {
                agg[0] = cv.take<char>(rows[0] * F * static_cast<int64_t>(xsz));
            }
        }
        // layer 2 of a 2-layer step: [self | agg] rows of 2H (the top launch writes
        // them dense, so the layer-2 weight gradient reads no self index)
        else agg[l - 1] = cv.take<float>(rows[l - 1] * (L == 2 ? 2 * H : H));
        h[l - 1] = (embed_out && l == L) ? embed_out : cv.take<float>(rows[l - 1] * H);
        if (l == L) T.last_emb = h[l - 1];
        if (l >= 2 && c.agg == GS_AGG_MAX) am[l - 1] = cv.take<int32_t>(rows[l - 1] * H);
    }
    float* demb = cv.take<float>(B * H);
    float* cls_ws = cv.take<float>(gs_cls_nll_ws_floats(B, H, c.n_classes));
    int64_t dw_need = 0, dx_rows = 0, dprev_rows = 0;
    for (int l = 1; l <= L; ++l) {
        dw_need = std::max(dw_need, gs_sage_linear_bwd_weight_ws(rows[l - 1], T.w_cols[l - 1], H));
        if (l >= 2) {
            dx_rows = std::max(dx_rows, rows[l - 1]);
            dprev_rows = std::max(dprev_rows, rows[l - 2]);
        }
    }
    char* dw_ws = cv.take<char>(dw_need);
    // the fused top path's dW_2 slabs outlive the layer-1 dW (their sum runs with layer 1's)
    const int64_t dw2_need = L == 2 ? gs_sage_linear_bwd_weight_ws(rows[1], T.w_cols[1], H) : 0;
    char* dw2_ws = dw2_need > 0 ? cv.take<char>(dw2_need) : nullptr;
    // the top launch's pair form writes dIn as two partials (dIn, then dIn + din2)
    const bool pair = !embed_out && roots && T.fuse_bwd && T.use_top && T.opt_top_pair && L == 2 &&
                      top_pair_supported(H, c.n_classes, c.gcn != 0);
    const int64_t din2 = pair ? dx_rows * 2 * H : 0;
    float* dIn = cv.take<float>(dx_rows * (c.gcn ? H : 2 * H) + din2);
    float* dbuf[2] = {cv.take<float>(dprev_rows * H), cv.take<float>(dprev_rows * H)};
    if (!ws) return cv.at + 256;
    GS_REQUIRE(cv.at <= ws_bytes, GS_EINVAL, "workspace too small");

    float* P = c.params;
    float* G = c.grads;
    // ---- forward (models.py:255-267)
    if (lowp && T.defer) {  // deferring: lp_buf(w1_cur) is cast once, then kept by the updates
        if (!T.lp_valid && !T.pending) {
            ok(gs_cast_f32_bf16(T.w1_buf(T.w1_cur), T.lp_buf(T.w1_cur), T.w_rows[0] * T.w_cols[0], st));
            T.lp_valid = true;
        }
    } else if (lowp && !(T.lp_keep && T.lp_valid)) {
        ok(gs_cast_f32_bf16(P + T.w_off[0], T.w1_lp, T.w_rows[0] * T.w_cols[0], st));
        T.lp_valid = T.lp_keep;
    }
    const int32_t* dst_L = fld(L, GS_PK_DST_IDS);
    // the layer-1 GEMMs' operands: X[dst_L] | agg, or the gather slot's dense
    // [self | agg] rows (GS_SELF_ROWS)
    const void* x1 = c.gcn ? nullptr : c.X;
    int64_t ldx1 = c.feat_ld, lda1 = F;
    const int32_t* sidx1 = dst_L;
    const void* a1 = agg[0];
    if (a1_slot >= 0 && T.self_rows) {
        const int64_t xsz1 = c.feat_dtype == GS_BF16 ? 2 : 4;
        a1 = static_cast<const char*>(agg[0]) + F * xsz1;
        lda1 = 2 * F;
        if (T.self_in_slot[a1_slot] && !c.gcn) {
            x1 = agg[0];
            ldx1 = 2 * F;
            sidx1 = nullptr;
        }
    }
    const void* W1 = lowp ? static_cast<const void*>(T.w1_lp) : static_cast<const void*>(P + T.w_off[0]);
    GS_REQUIRE(!T.defer || !embed_out, GS_EINVAL, "deferred update: unsupported step");
    bool pend = T.defer && T.pending;
    if (pend && !(T.pend_np[0] >= 1 && T.pend_np[0] <= 512 && T.pend_np[1] >= 1 && T.pend_np[1] <= 512 &&
                  linear_fwd_wide_ok(static_cast<gs_dtype>(c.feat_dtype), F, x1, ldx1, a1, lda1,
                                     lowp ? static_cast<const void*>(T.lp_buf(T.w1_cur ^ 1))
                                          : static_cast<const void*>(T.w1_buf(T.w1_cur ^ 1))))) {
        // the forward folds at most 512 partials per group, and only the wide
        // (16-B load) forward applies a pending update: apply it on its own
        trainer_defer_update(&T, false, st);
        trainer_defer_update(&T, true, st);
        pend = false;
    }
    if (T.defer) {
        const int wb = pend ? T.w1_cur ^ 1 : T.w1_cur;
        W1 = lowp ? static_cast<const void*>(T.lp_buf(wb)) : static_cast<const void*>(T.w1_buf(wb));
        if (pend) {  // the previous step's clip + SGD, applied by this forward launch
            FwdSpec sp;
            sp.on = 1;
            sp.S = T.w1_buf(T.w1_cur ^ 1);
            sp.P = T.w1_buf(T.w1_cur);
            sp.Wn = T.w1_buf(T.w1_cur ^ 1);
            if (lowp) {
                sp.S_lp = T.lp_buf(T.w1_cur ^ 1);
                sp.Wn_lp = T.lp_buf(T.w1_cur ^ 1);
            }
            sp.G1 = G + T.w_off[0];
            sp.part0 = T.pend_part;
            sp.part1 = T.pend_part + T.pend_pstride;
            sp.np0 = T.pend_np[0];
            sp.np1 = T.pend_np[1];
            sp.lr = c.lr;
            sp.max_norm = c.max_norm;
            sp.scale = T.pend_scale;
            sp.p = P;
            sp.g = G;
            sp.up_lo = T.w_off[0] + T.w_rows[0] * T.w_cols[0];
            sp.up_hi = T.total;
            sp.grp1_lo = T.cls_w_off;
            g_fwd_spec = sp;
        }
    }
    if (a1_slot < 0) gather1(T, pack, hop_sizes, offsets, agg[0], st);
    {
        const bool armed = timed_arm(T, 1);
        ok(gs_sage_linear_fwd(static_cast<gs_dtype>(c.feat_dtype), rows[0], F, H, x1, ldx1, sidx1, a1, lda1, W1, h[0],
                              H, 1, st));
        g_launch_events = {};  // an alternative kernel that does not time leaves it armed
        timed_done(T, 1, armed);
        if (pend) {  // the launch took the pending update: W1 is now the other buffer
            GS_REQUIRE(!g_fwd_spec.on, GS_EINVAL, "the forward launch did not take the pending update");
            T.w1_cur ^= 1;
            T.pending = false;
        }
    }
    // a 2-layer training step runs layer 2, the loss head and layer 2's dIn in
    // one launch (top.hip) inside the fused backward below
    const bool top = !embed_out && roots && T.fuse_bwd && T.use_top && L == 2 &&
                     top_supported(H, c.n_classes, c.gcn != 0);
    for (int l = 2; l <= L && !top; ++l) {
        const int j = L - l + 1;
        ok(gs_agg_fwd(static_cast<gs_agg>(c.agg), GS_F32, h[l - 2], H, H, rows[l - 1], fld(j, GS_PK_NBR_PTR),
                      fld(j, GS_PK_NBR), nullptr, nullptr, nullptr, 0, agg[l - 1], GS_F32, H, am[l - 1], st));
        ok(gs_sage_linear_fwd(GS_F32, rows[l - 1], H, H, c.gcn ? nullptr : h[l - 2], H, fld(j, GS_PK_SELF),
                              agg[l - 1], H, P + T.w_off[l - 1], h[l - 1], H, 1, st));
    }
    if (embed_out) return cv.at;  // inference: no loss head, no backward
    T.norm_ready = false;
    // ---- fused backward (bwd.hip): same kernels and summation order as the
    // sequence below, two launches per layer >= 2 instead of five
    if (T.fuse_bwd && L >= 2) {
        std::vector<LayerBwd> lb;
        int flip_f = 0;
        bool fusable = true;
        for (int l = L; l >= 2; --l) {
            const int j = L - l + 1;
            LayerBwd a{};
            a.n = rows[l - 1];
            a.fin = H;
            a.H = H;
            a.Xs = c.gcn ? nullptr : h[l - 2];
            a.ldxs = H;
            a.sidx = fld(j, GS_PK_SELF);
            a.A = static_cast<const float*>(agg[l - 1]);
            if (top && l == L) {  // the top launch's dense [self | agg] rows: no self index
                a.Xs = static_cast<const float*>(agg[l - 1]);
                a.ldxs = 2 * H;
                a.sidx = nullptr;
                a.A = static_cast<const float*>(agg[l - 1]) + H;
                a.lda = 2 * H;
            }
            a.dZ = l == L ? demb : dbuf[flip_f ^ 1];
            a.W = P + T.w_off[l - 1];
            a.dW = G + T.w_off[l - 1];
            a.slabs = reinterpret_cast<float*>(dw_ws);
            a.slab_bytes = dw_need;
            a.dIn = dIn;
            a.agg = c.agg;
            a.n_src = rows[l - 2];
            a.tptr = fld(j, GS_PK_TPTR);
            a.tidx = fld(j, GS_PK_TIDX);
            a.ptr = fld(j, GS_PK_NBR_PTR);
            a.argmax = am[l - 1];
            a.Hprev = h[l - 2];
            a.dH = dbuf[flip_f];
            if (top && l == L && a1_slot >= 0 && T.rec_ready[a1_slot])  // the side stream's records of hop 1's lists
                a.trec = reinterpret_cast<const int4*>(T.rec_slot[a1_slot]);
            flip_f ^= 1;
            fusable = fusable && layer_bwd_fusable(a);
            lb.push_back(a);
        }
        GS_REQUIRE(!top || fusable, GS_EINVAL, "top launch needs the fused backward");
        if (fusable) {
            int cls_rows;
            if (top) {
                const bool armed = timed_arm(T, 3);
                const bool tids = a1_slot >= 0 && T.top_ready[a1_slot];
                if (pair) {
                    top_pair_reserve(T, B, st);
                    cls_rows = top_pair_fwd_bwd(c.agg, B, c.n_classes, h[0], fld(1, GS_PK_NBR_PTR), fld(1, GS_PK_NBR),
                                                fld(1, GS_PK_SELF), P + T.w_off[1], P + T.cls_w_off, P + T.cls_b_off,
                                                c.labels, roots, static_cast<float*>(agg[1]), am[1], h[1], demb, dIn,
                                                dIn + din2, cls_ws, T.xch, ++T.xch_epoch == 0 ? ++T.xch_epoch : T.xch_epoch,
                                                T.xch_fail, st, tids ? T.top_slot[a1_slot] : nullptr,
                                                tids ? T.top_k : 0);
                    lb[0].din_off2 = din2;
                } else {
                    cls_rows = top_fwd_bwd(c.agg, B, c.n_classes, h[0], fld(1, GS_PK_NBR_PTR), fld(1, GS_PK_NBR),
                                           fld(1, GS_PK_SELF), P + T.w_off[1], P + T.cls_w_off, P + T.cls_b_off,
                                           c.labels, roots, static_cast<float*>(agg[1]), am[1], h[1], demb, dIn, cls_ws,
                                           st, tids ? T.top_slot[a1_slot] : nullptr, tids ? T.top_k : 0);
                }
                timed_done(T, 3, armed);
                lb[0].din_ready = true;
            } else {
                cls_rows = cls_rows_launch(B, H, c.n_classes, h[L - 1], P + T.cls_w_off, P + T.cls_b_off, c.labels,
                                           roots, 1, demb, cls_ws, st);
            }
            const ClsReduce cr{B, H, c.n_classes, cls_rows, cls_ws, G + T.cls_w_off, G + T.cls_b_off, loss,
                               T.norm_part + T.pstride};
            const int64_t K1 = T.w_cols[0];
            // top path, 2 layers, no bucketed all-reduce hook: one backward launch for
            // layer 2 and its slab sum beside layer 1's (same sums, partials, order)
            const bool defer = top && lb.size() == 1 && !T.upper_hook && dw2_ws &&
                               sum_slabs_pair_ok(H * K1, H * T.w_cols[1]);
            int np = 0;
            bool parts = true;
            SlabSum d2{};
            if (defer) {
                lb[0].slabs = reinterpret_cast<float*>(dw2_ws);
                lb[0].slab_bytes = dw2_need;
                np = layer_bwd_top(lb[0], cr, &d2, st);
                parts = np > 0;
            } else {
                for (size_t i = 0; i < lb.size(); ++i) {
                    const int n = layer_bwd(lb[i], i == 0 ? &cr : nullptr, T.norm_part + np, st);
                    parts = parts && n > 0;
                    np += n;
                }
                if (T.upper_hook) T.upper_hook(st);
            }
            if (!defer && T.w1_chunk_hook && T.w1_chunks > 1 && H % (64 * T.w1_chunks) == 0) {
                // dW1 in row chunks, each summed and handed to the hook (its
                // all-reduce then runs under the next chunk's GEMM); the clip
                // of the communicator path recomputes the norm from the
                // reduced gradient, so no norm partials are kept
                const int64_t Hc = H / T.w1_chunks;
                for (int q = 0; q < T.w1_chunks; ++q) {
                    const int64_t h0 = q * Hc;
                    float* dWq = G + T.w_off[0] + h0 * K1;
                    const int Sq = linear_dw_slabs(static_cast<gs_dtype>(c.feat_dtype), rows[0], F, Hc, x1, ldx1,
                                                   sidx1, a1, lda1, lb.back().dH + h0, h[0] + h0, H, 0, dWq, dw_ws,
                                                   dw_need, st, H, kDw1Phases);
                    if (Sq > 1) sum_slabs_launch(reinterpret_cast<const float*>(dw_ws), Sq, Hc * K1, dWq, nullptr, st);
                    T.w1_chunk_hook(st, T.w_off[0] + h0 * K1, Hc * K1);
                }
                g_launch_events = {};
                T.npart[0] = 0;
                T.npart[1] = 0;
                T.norm_ready = false;
                return cv.at;
            }
            const bool armed = timed_arm(T, 2);
            const int S1 = linear_dw_slabs(static_cast<gs_dtype>(c.feat_dtype), rows[0], F, H, x1, ldx1, sidx1, a1,
                                           lda1, lb.back().dH, h[0], H, 0, G + T.w_off[0], dw_ws, dw_need, st, -1,
                                           kDw1Phases);
            g_launch_events = {};
            timed_done(T, 2, armed);
            const float* s1_src = S1 > 1 ? reinterpret_cast<const float*>(dw_ws) : nullptr;
            const int s1_n = S1;
            const int n_cls = cls_reduce_grid(c.n_classes, H);
            if (defer && S1 > 1) {
                d2.part = T.norm_part;
                // deferred update: this launch also writes W1's update for clip
                // coefficient 1 (and carries the done flag); the clip + SGD
                // itself is left to the next forward
                const bool spec = T.defer && !T.defer_comm && parts && np + sum_slabs_grid(H * K1) <= T.pstride &&
                                  n_cls <= T.pstride;
                const bool armed = timed_arm(T, 4);
                np += sum_slabs_pair_launch(SlabSum{s1_src, s1_n, H * K1, G + T.w_off[0], T.norm_part + np}, d2, st,
                                            spec ? T.w1_buf(T.w1_cur) : nullptr,
                                            spec ? T.w1_buf(T.w1_cur ^ 1) : nullptr, c.lr,
                                            spec && lowp ? T.lp_buf(T.w1_cur ^ 1) : nullptr);
                timed_done(T, 4, armed);
                T.pending = spec;
                if (spec) {
                    T.pend_part = T.norm_part;
                    T.pend_pstride = T.pstride;
                    T.pend_np[0] = np;
                    T.pend_np[1] = n_cls;
                    T.pend_scale = 1.f;
                }
            } else if (defer) {
                if (d2.S > 1) sum_slabs_launch(d2.slabs, d2.S, d2.len, d2.out, nullptr, st);
                parts = false;
            } else if (S1 > 1) {
                np += sum_slabs_launch(s1_src, s1_n, H * K1, G + T.w_off[0], T.norm_part + np, st);
            } else {
                parts = false;
            }
            T.npart[0] = np;
            T.npart[1] = n_cls;
            T.norm_ready = parts && np <= T.pstride && T.npart[1] <= T.pstride;
            return cv.at;
        }
    }
    // ---- loss head (models.py:8-27, utils.py:159-164); labels gathered through
    // the roots, and demb comes back already masked by relu'(h_L), i.e. dZ_L
    ok(gs_cls_nll_fwd_bwd(B, H, c.n_classes, h[L - 1], P + T.cls_w_off, P + T.cls_b_off, c.labels, roots, 1, loss,
                          demb, G + T.cls_w_off, G + T.cls_b_off, cls_ws, st));
    // ---- backward (utils.py:184); every dH below is pre-masked, so relu = 0
    const float* dH = demb;
    const int relu = 0;
    int flip = 0;
    for (int l = L; l >= 1; --l) {
        const int j = L - l + 1;
        const bool first = l == 1;
        const void* x_in = first ? x1 : (c.gcn ? nullptr : h[l - 2]);
        const int32_t* sidx = first ? sidx1 : fld(j, GS_PK_SELF);
        const int64_t fin = in_dim[l - 1], ldx = first ? ldx1 : H;
        if (first && L >= 2 && T.upper_hook) T.upper_hook(st);
        {  // the fused path's slabs: layer 1 in kDw1Phases row phases, layers >= 2 in one
            const int64_t Kl = x_in ? 2 * fin : fin;
            const int Sl = linear_dw_slabs(first ? static_cast<gs_dtype>(c.feat_dtype) : GS_F32, rows[l - 1], fin, H,
                                           x_in, ldx, sidx, first ? a1 : agg[l - 1], first ? lda1 : fin, dH, h[l - 1],
                                           H, relu, G + T.w_off[l - 1], dw_ws, dw_need, st, -1,
                                           first ? kDw1Phases : 1);
            if (Sl > 1) sum_slabs_launch(reinterpret_cast<const float*>(dw_ws), Sl, H * Kl, G + T.w_off[l - 1], nullptr,
                                         st);
        }
        if (first) break;
        const int64_t ldd = c.gcn ? H : 2 * H;
        float* dSelf = c.gcn ? nullptr : dIn;
        float* dA = c.gcn ? dIn : dIn + H;
        ok(gs_sage_linear_bwd_input(rows[l - 1], H, H, dH, h[l - 1], H, relu, P + T.w_off[l - 1], dSelf, dA, ldd,
                                    st));
        float* dprev = dbuf[flip];
        flip ^= 1;
        ok(gs_agg_bwd(static_cast<gs_agg>(c.agg), rows[l - 2], H, fld(j, GS_PK_TPTR), fld(j, GS_PK_TIDX),
                      fld(j, GS_PK_NBR_PTR), dA, dSelf, ldd, am[l - 1], h[l - 2], H, dprev, st));
        dH = dprev;  // agg_bwd masks by relu'(h_{l-1})
    }
    return cv.at;
}

// The parity capture of one finished training step (gs_trainer_capture).
static void capture_step(gs_trainer& T, int64_t B, hipStream_t st) {
    auto& c = T.cap;
    if (c.n >= c.max_steps || (!c.emb && !c.grads)) return;
    if (c.emb) {
        GS_REQUIRE(B * T.cfg.hidden <= c.emb_stride, GS_EINVAL, "capture: batch larger than the embedding stride");
        GS_REQUIRE(hipMemcpyAsync(c.emb + c.n * c.emb_stride, T.last_emb, B * T.cfg.hidden * sizeof(float),
                                  hipMemcpyDeviceToDevice, st) == hipSuccess,
                   GS_EHIP, "hipMemcpyAsync(capture)");
    }
    if (c.grads)
        GS_REQUIRE(hipMemcpyAsync(c.grads + c.n * T.total, T.cfg.grads, T.total * sizeof(float),
                                  hipMemcpyDeviceToDevice, st) == hipSuccess,
                   GS_EHIP, "hipMemcpyAsync(capture)");
    ++c.n;
}

void trainer_set_upper_hook(gs_trainer* t, std::function<void(hipStream_t)> hook) { t->upper_hook = std::move(hook); }
void trainer_set_w1_chunk_hook(gs_trainer* t, int chunks, std::function<void(hipStream_t, int64_t, int64_t)> hook) {
    t->w1_chunks = hook ? std::max(1, chunks) : 1;
    t->w1_chunk_hook = std::move(hook);
}

// the pair form's exchange buffer for batches of up to B roots (grown on
// demand, zeroed on the stream when allocated) and its give-up flag
void top_pair_reserve(gs_trainer& t, int64_t B, hipStream_t st) {
    const int64_t words = top_pair_xch_words(B);
    if (words > t.xch_quads) {
        if (t.xch) GS_REQUIRE(hipFree(t.xch) == hipSuccess, GS_EHIP, "hipFree");
        t.xch = nullptr;
        GS_REQUIRE(hipMalloc(&t.xch, words * 8) == hipSuccess, GS_ENOMEM, "hipMalloc(top exchange)");
        GS_REQUIRE(hipMemsetAsync(t.xch, 0, words * 8, st) == hipSuccess, GS_EHIP, "hipMemsetAsync");
        t.xch_quads = words;
    }
    if (!t.xch_fail) {
        GS_REQUIRE(hipMalloc(&t.xch_fail, 16) == hipSuccess, GS_ENOMEM, "hipMalloc(top exchange flag)");
        GS_REQUIRE(hipMemsetAsync(t.xch_fail, 0, 16, st) == hipSuccess, GS_EHIP, "hipMemsetAsync");
    }
}

void trainer_reserve_top(gs_trainer* t, int64_t B, int32_t tk) {
    if (t->cfg.n_layers != 2 || t->cfg.gcn || tk < 1 || tk > 31 || B < 1) return;
    if (B <= t->top_rows && tk == t->top_k) return;
    for (int32_t*& p : t->top_slot) {
        if (p) GS_REQUIRE(hipFree(p) == hipSuccess, GS_EHIP, "hipFree");
        p = nullptr;
        GS_REQUIRE(hipMalloc(&p, std::max<int64_t>(B * (tk + 1) * 4, 256)) == hipSuccess, GS_ENOMEM,
                   "hipMalloc(top records)");
    }
    for (bool& r : t->top_ready) r = false;
    t->top_rows = B;
    t->top_k = tk;
    // the backward's records for up to a1_rows layer-1 rows (gs_trainer_gather_reserve first)
    for (int32_t*& p : t->rec_slot) {
        if (p) GS_REQUIRE(hipFree(p) == hipSuccess, GS_EHIP, "hipFree");
        p = nullptr;
        GS_REQUIRE(hipMalloc(&p, std::max<int64_t>(t->a1_rows * 8 * 4, 256)) == hipSuccess, GS_ENOMEM,
                   "hipMalloc(backward records)");
    }
    for (bool& r : t->rec_ready) r = false;
    t->rec_rows = t->a1_rows;
}

int64_t trainer_w1_floats(const gs_trainer* t) { return t->w_rows[0] * t->w_cols[0]; }

}  // namespace gs

namespace {
// The SGD launch that follows also writes the bf16 W1 (runner loops only).
struct ShadowArm {
    gs_trainer* t;
    explicit ShadowArm(gs_trainer* t_) : t(t_) {
        t->lp_valid = false;
        if (t->lp_keep && t->w1_lp)
            gs::g_lowp_shadow = {t->w1_lp, t->w_off[0], t->w_off[0] + t->w_rows[0] * t->w_cols[0]};
    }
    void done() { t->lp_valid = t->lp_keep && t->w1_lp; }
    ~ShadowArm() { gs::g_lowp_shadow = {}; }
};
}  // namespace

namespace gs {
void trainer_keep_lowp(gs_trainer* t, bool keep) {
    t->lp_keep = keep;
    t->lp_valid = false;
}


// W1 back in the flat params (a pending update stays pending: its S and P
// buffers are then the flat W1 and w1_alt, or it is finalised by the caller).
static void w1_home(gs_trainer* t, hipStream_t st) {
    if (t->w1_cur == 0) return;
    GS_REQUIRE(!t->pending, GS_EINVAL, "W1 moved with an update pending");
    const int64_t n = t->w_rows[0] * t->w_cols[0];
    GS_REQUIRE(hipMemcpyAsync(t->w1_buf(0), t->w1_alt, n * sizeof(float), hipMemcpyDeviceToDevice, st) == hipSuccess,
               GS_EHIP, "hipMemcpyAsync(W1)");
    t->w1_cur = 0;
}

bool trainer_defer_update(gs_trainer* t, bool on, hipStream_t st, bool comm) {
    if (!on) {
        if (t->pending) {  // the last step's clip + SGD: the flat params become what sgd4 would leave
            FwdSpec sp;
            sp.on = 1;
            sp.S = t->w1_buf(t->w1_cur ^ 1);
            sp.P = t->w1_buf(t->w1_cur);
            sp.G1 = t->cfg.grads + t->w_off[0];
            sp.part0 = t->pend_part;
            sp.part1 = t->pend_part + t->pend_pstride;
            sp.np0 = t->pend_np[0];
            sp.np1 = t->pend_np[1];
            sp.lr = t->cfg.lr;
            sp.max_norm = t->cfg.max_norm;
            sp.scale = t->pend_scale;
            sp.p = t->cfg.params;
            sp.g = t->cfg.grads;
            sp.up_lo = t->w_off[0] + t->w_rows[0] * t->w_cols[0];
            sp.up_hi = t->total;
            sp.grp1_lo = t->cls_w_off;
            spec_finalize_launch(sp, t->w1_buf(0), t->w_rows[0] * t->w_cols[0], st);
            t->pending = false;
            t->w1_cur = 0;
        }
        w1_home(t, st);
        t->defer = false;
        t->defer_comm = false;
        t->norm_ready = false;
        t->lp_valid = false;  // the next bf16 forward casts the flat W1 again
        return false;
    }
    const gs_trainer_config& c = t->cfg;
    const int64_t n1 = t->w_rows[0] * t->w_cols[0];
    // the pending update is applied by the wide (16-B load) layer-1 forward:
    // its feature rows must take 16-B loads (run_step re-checks each step's
    // operands and applies the update on its own where they do not)
    const int64_t epv = c.feat_dtype == GS_F32 ? 4 : 8;
    const bool ok = t->opt_defer && (c.feat_dtype == GS_F32 || (c.feat_dtype == GS_BF16 && t->w1_lp)) &&
                    t->fuse_bwd && t->use_top && c.n_layers == 2 && !c.gcn &&
                    (comm || (!t->upper_hook && !t->w1_chunk_hook)) && n1 % 4 == 0 &&
                    c.feat_dim % epv == 0 && c.feat_ld % epv == 0 && aligned16(c.X) &&
                    t->cls_w_off % 4 == 0 && t->total % 4 == 0 && aligned16(c.params) && aligned16(c.grads);
    if (!ok) return false;
    if (!t->w1_alt)
        GS_REQUIRE(hipMalloc(&t->w1_alt, n1 * sizeof(float)) == hipSuccess, GS_ENOMEM, "hipMalloc(W1 buffer)");
    if (c.feat_dtype == GS_BF16 && !t->w1_lp_alt)
        GS_REQUIRE(hipMalloc(&t->w1_lp_alt, n1 * sizeof(uint16_t)) == hipSuccess, GS_ENOMEM, "hipMalloc(bf16 W1)");
    t->lp_valid = false;  // the first forward casts W1 into lp_buf(0)
    t->defer = true;
    t->defer_comm = comm;
    t->pending = false;
    t->w1_cur = 0;
    return true;
}

}  // namespace gs

extern "C" {

int gs_trainer_create(const gs_trainer_config* cfg, gs_trainer** out) {
    GS_API_BEGIN
    GS_REQUIRE(cfg && out, GS_EINVAL, "NULL argument");
    GS_REQUIRE(cfg->n_layers >= 1 && cfg->n_layers <= GS_MAX_HOPS, GS_EINVAL, "n_layers out of range");
    GS_REQUIRE(cfg->hidden >= 16 && cfg->hidden <= 256 && cfg->hidden % 16 == 0, GS_EINVAL, "bad hidden size");
    GS_REQUIRE(cfg->n_classes >= 1 && cfg->feat_dim >= 1 && cfg->feat_ld >= cfg->feat_dim, GS_EINVAL, "bad dims");
    GS_REQUIRE(cfg->X && cfg->col && cfg->labels && cfg->params && cfg->grads, GS_EINVAL,
               "NULL device pointer");
    auto* T = new gs_trainer();
    T->cfg = *cfg;
    int64_t at = 0;
    for (int l = 1; l <= cfg->n_layers; ++l) {
        const int64_t in = l == 1 ? cfg->feat_dim : cfg->hidden;
        T->w_off.push_back(at);
        T->w_rows.push_back(cfg->hidden);
        T->w_cols.push_back(cfg->gcn ? in : 2 * in);
        at += cfg->hidden * T->w_cols.back();
    }
    T->cls_w_off = at;
    at += static_cast<int64_t>(cfg->n_classes) * cfg->hidden;
    T->cls_b_off = at;
    at += cfg->n_classes;
    T->total = at;
    {
        int64_t np = 0;
        for (int l = 1; l <= cfg->n_layers; ++l) np += gs::sum_slabs_grid(cfg->hidden * T->w_cols[l - 1]);
        np = std::max<int64_t>({np, gs::cls_reduce_grid(cfg->n_classes, cfg->hidden), 64});
        T->pstride = static_cast<int>((np + 63) / 64 * 64);
        if (hipMalloc(&T->norm_part, 2 * T->pstride * sizeof(float)) != hipSuccess) {
            delete T;
            gs::fail(GS_ENOMEM, "hipMalloc(norm partials)");
        }
        if (cfg->feat_dtype == GS_BF16 &&
            hipMalloc(&T->w1_lp, T->w_rows[0] * T->w_cols[0] * sizeof(uint16_t)) != hipSuccess) {
            delete T;
            gs::fail(GS_ENOMEM, "hipMalloc(bf16 W1)");
        }
    }
    *out = T;
    GS_API_END
}

void gs_trainer_destroy(gs_trainer* t) { delete t; }

int64_t gs_trainer_n_params(const gs_trainer* t) { return t ? t->total : -1; }

float* gs_trainer_grads(const gs_trainer* t) { return t ? t->cfg.grads : nullptr; }

int gs_trainer_set_option(gs_trainer* t, int32_t opt, int32_t value) {
    GS_API_BEGIN
    GS_REQUIRE(t, GS_EINVAL, "NULL argument");
    GS_REQUIRE(!t->defer && !t->pending, GS_EINVAL, "options cannot change inside a runner loop");
    const bool on = value != 0;
    switch (opt) {
        case GS_TOPT_FUSED_BWD: t->fuse_bwd = on; break;
        case GS_TOPT_TOP_LAUNCH: t->use_top = on; break;
        case GS_TOPT_SELF_ROWS: t->want_self_rows = on; break;
        case GS_TOPT_DEFER_UPDATE: t->opt_defer = on; break;
        case GS_TOPT_TOP_PAIR: t->opt_top_pair = on; break;
        default: GS_REQUIRE(false, GS_EINVAL, "unknown trainer option");
    }
    GS_API_END
}

int64_t gs_trainer_ws_bytes(gs_trainer* t, const int64_t* hop_sizes) {
    try {
        std::vector<int64_t> off(GS_MAX_HOPS * GS_PK_NFIELDS, 0);
        return gs::run_step(*t, nullptr, hop_sizes, off.data(), nullptr, hop_sizes[0], nullptr, 0, nullptr,
                            nullptr);
    } catch (const gs::Error& e) {
        gs::set_error(e.what());
        return -1;
    }
}

int gs_trainer_forward_backward(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                                const int64_t* offsets, const int32_t* roots, int64_t n_roots, void* ws,
                                int64_t ws_bytes, float* loss, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && pack && hop_sizes && offsets && roots && ws && loss, GS_EINVAL, "NULL argument");
    gs::run_step(*t, pack, hop_sizes, offsets, roots, n_roots, static_cast<char*>(ws), ws_bytes, loss,
                 gs::as_stream(stream));
    gs::capture_step(*t, n_roots, gs::as_stream(stream));
    GS_API_END
}

int gs_trainer_capture(gs_trainer* t, float* emb, int64_t emb_stride, float* grads, int64_t max_steps) {
    GS_API_BEGIN
    GS_REQUIRE(t && max_steps >= 0 && (!emb || emb_stride >= t->cfg.hidden), GS_EINVAL, "bad arguments");
    t->cap = {};
    t->cap.emb = emb;
    t->cap.emb_stride = emb_stride;
    t->cap.grads = grads;
    t->cap.max_steps = max_steps;
    GS_API_END
}

int64_t gs_trainer_captured(const gs_trainer* t) { return t ? t->cap.n : -1; }

int gs_trainer_gather_reserve(gs_trainer* t, int64_t max_rows, int32_t max_fanout) {
    GS_API_BEGIN
    GS_REQUIRE(t && max_rows >= 0 && max_fanout >= 0, GS_EINVAL, "bad arguments");
    const bool self_rows = t->want_self_rows && !t->cfg.gcn && t->cfg.n_layers >= 1;
    if (max_rows <= t->a1_rows && max_fanout <= t->k_ids && self_rows == t->self_rows) return GS_OK;
    max_rows = std::max(max_rows, t->a1_rows);
    t->self_rows = self_rows;
    for (bool& b : t->self_in_slot) b = false;
    const int64_t bytes = max_rows * t->cfg.feat_dim * (self_rows ? 2 : 1) * (t->cfg.feat_dtype == GS_BF16 ? 2 : 4);
    for (void*& p : t->a1_slot) {
        if (p) GS_REQUIRE(hipFree(p) == hipSuccess, GS_EHIP, "hipFree");
        p = nullptr;
        GS_REQUIRE(hipMalloc(&p, std::max<int64_t>(bytes, 256)) == hipSuccess, GS_ENOMEM, "hipMalloc(gather slot)");
    }
    for (int32_t*& p : t->ids_slot) {
        if (p) GS_REQUIRE(hipFree(p) == hipSuccess, GS_EHIP, "hipFree");
        p = nullptr;
    }
    t->k_ids = 0;
    if (max_fanout > 0) {
        GS_REQUIRE(max_rows * max_fanout < (int64_t(1) << 31), GS_EINVAL, "gather slot too large for int32 ids");
        for (int32_t*& p : t->ids_slot)
            GS_REQUIRE(hipMalloc(&p, std::max<int64_t>(max_rows * max_fanout * 4, 256)) == hipSuccess, GS_ENOMEM,
                       "hipMalloc(gather ids)");
        t->k_ids = max_fanout;
    }
    t->a1_rows = max_rows;
    GS_API_END
}

int gs_trainer_gather(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes, const int64_t* offsets,
                      int32_t slot, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && pack && hop_sizes && offsets && slot >= 0 && slot < gs_trainer::kSlots, GS_EINVAL,
               "bad arguments");
    const int L = t->cfg.n_layers;
    GS_REQUIRE(hop_sizes[4 * (L - 1)] <= t->a1_rows && t->a1_slot[slot], GS_EINVAL,
               "gather slot too small (gs_trainer_gather_reserve)");
    const int64_t n_dst = hop_sizes[4 * (L - 1)], n_pos = hop_sizes[4 * (L - 1) + 1];
    if (t->k_ids > 0 && n_pos <= n_dst * t->k_ids) {  // every neighbourhood fits k_ids slots
        gs::gather1_ids(*t, pack, hop_sizes, offsets, slot, gs::as_stream(stream));
    } else if (t->self_rows) {  // the agg half only: the GEMMs gather the self rows themselves
        const int64_t F = t->cfg.feat_dim, xsz = t->cfg.feat_dtype == GS_BF16 ? 2 : 4;
        gs::gather1(*t, pack, hop_sizes, offsets, static_cast<char*>(t->a1_slot[slot]) + F * xsz,
                    gs::as_stream(stream), 2 * F);
        t->self_in_slot[slot] = false;
    } else {
        gs::gather1(*t, pack, hop_sizes, offsets, t->a1_slot[slot], gs::as_stream(stream));
    }
    GS_API_END
}

int gs_trainer_forward_backward_gathered(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                                         const int64_t* offsets, const int32_t* roots, int64_t n_roots,
                                         int32_t slot, void* ws, int64_t ws_bytes, float* loss, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && pack && hop_sizes && offsets && roots && ws && loss && slot >= 0 && slot < gs_trainer::kSlots,
               GS_EINVAL, "bad arguments");
    gs::run_step(*t, pack, hop_sizes, offsets, roots, n_roots, static_cast<char*>(ws), ws_bytes, loss,
                 gs::as_stream(stream), slot);
    gs::capture_step(*t, n_roots, gs::as_stream(stream));
    GS_API_END
}

int gs_trainer_forward(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes, const int64_t* offsets,
                       void* ws, int64_t ws_bytes, float* out, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && pack && hop_sizes && offsets && ws && out, GS_EINVAL, "NULL argument");
    gs::run_step(*t, pack, hop_sizes, offsets, nullptr, hop_sizes[0], static_cast<char*>(ws), ws_bytes, nullptr,
                 gs::as_stream(stream), -1, out);
    GS_API_END
}

int gs_trainer_forward_gathered(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                                const int64_t* offsets, int32_t slot, void* ws, int64_t ws_bytes, float* out,
                                void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && pack && hop_sizes && offsets && ws && out && slot >= 0 && slot < gs_trainer::kSlots, GS_EINVAL,
               "bad arguments");
    gs::run_step(*t, pack, hop_sizes, offsets, nullptr, hop_sizes[0], static_cast<char*>(ws), ws_bytes, nullptr,
                 gs::as_stream(stream), slot, out);
    GS_API_END
}

int gs_trainer_time_kernels(gs_trainer* t, int32_t site_mask, int64_t capacity) {
    return gs_trainer_time_kernels_every(t, site_mask, capacity, 1);
}

int gs_trainer_time_kernels_every(gs_trainer* t, int32_t site_mask, int64_t capacity, int64_t every) {
    GS_API_BEGIN
    GS_REQUIRE(t && capacity >= 0 && every >= 1, GS_EINVAL, "bad arguments");
    for (int s = 0; s < gs_trainer::kSites; ++s) {
        auto& tm = t->timer[s];
        for (auto e : tm.ev0) (void)hipEventDestroy(e);
        for (auto e : tm.ev1) (void)hipEventDestroy(e);
        const int64_t cap = (site_mask >> s) & 1 ? capacity : 0;
        tm.ev0.assign(cap, nullptr);
        tm.ev1.assign(cap, nullptr);
        if (tm.st0) (void)hipFree(tm.st0);
        tm.st0 = tm.st1 = nullptr;
        tm.stamped.assign(cap, 0);
        if (s >= 1 && cap > 0) {  // span stamps (forward, dW, top, slab sum)
            const int64_t words = cap * gs::kStampBlocks;
            GS_REQUIRE(hipMalloc(&tm.st0, 2 * words * sizeof(unsigned long long)) == hipSuccess, GS_ENOMEM,
                       "hipMalloc(timer stamps)");
            tm.st1 = tm.st0 + words;
            GS_REQUIRE(hipMemset(tm.st0, 0, 2 * words * sizeof(unsigned long long)) == hipSuccess, GS_EHIP,
                       "hipMemset(timer stamps)");
        }
        for (int64_t i = 0; i < cap; ++i)
            GS_REQUIRE(hipEventCreateWithFlags(&tm.ev0[i], gs::timer_event_flags()) == hipSuccess &&
                           hipEventCreateWithFlags(&tm.ev1[i], gs::timer_event_flags()) == hipSuccess,
                       GS_EHIP, "hipEventCreate");
        tm.n = 0;
        tm.every = every;
        tm.calls = 0;
        tm.kernel.clear();
    }
    GS_API_END
}

int gs_trainer_time_agg(gs_trainer* t, int64_t capacity) { return gs_trainer_time_kernels(t, 1, capacity); }

int64_t gs_trainer_kernel_times(gs_trainer* t, int32_t site, float* ms, int64_t cap) {
    if (!t || !ms || site < 0 || site >= gs_trainer::kSites) return -1;
    auto& tm = t->timer[site];
    const int64_t n = std::min(cap, tm.n);
    std::vector<unsigned long long> a, b;
    const int64_t W = gs::kStampBlocks;
    if (tm.st0 && n > 0) {
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        a.resize(n * W);
        b.resize(n * W);
        if (hipMemcpy(a.data(), tm.st0, n * W * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(b.data(), tm.st1, n * W * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (tm.st0 && tm.stamped[i]) {  // the kernel's own span: min start .. max end, 100 MHz ticks
            unsigned long long lo = ~0ull, hi = 0;
            for (int64_t w = 0; w < W; ++w) {
                if (a[i * W + w]) lo = std::min(lo, a[i * W + w]);
                hi = std::max(hi, b[i * W + w]);
            }
            if (hi == 0 || lo == ~0ull || hi < lo) return -1;
            ms[i] = static_cast<float>(static_cast<double>(hi - lo) * 1e-5);
            continue;
        }
        if (hipEventSynchronize(tm.ev1[i]) != hipSuccess || hipEventElapsedTime(&ms[i], tm.ev0[i], tm.ev1[i]) != hipSuccess)
            return -1;
    }
    return n;
}

int64_t gs_trainer_kernel_stamps(gs_trainer* t, int32_t site, int64_t launch, uint64_t* start, uint64_t* end) {
    if (!t || !start || !end || site < 0 || site >= gs_trainer::kSites) return -1;
    auto& tm = t->timer[site];
    if (!tm.st0 || launch < 0 || launch >= tm.n) return 0;
    const int64_t W = gs::kStampBlocks;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(start, tm.st0 + launch * W, W * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(end, tm.st1 + launch * W, W * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return W;
}

int64_t gs_trainer_kernel_block_stats(gs_trainer* t, int32_t site, float* us4, int64_t cap) {
    if (!t || !us4 || site < 0 || site >= gs_trainer::kSites) return -1;
    auto& tm = t->timer[site];
    const int64_t n = std::min(cap, tm.n);
    const int64_t W = gs::kStampBlocks;
    if (n <= 0) return 0;
    if (!tm.st0) {  // an event-timed site
        std::fill(us4, us4 + 4 * n, -1.f);
        return n;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::vector<unsigned long long> a(n * W), b(n * W);
    if (hipMemcpy(a.data(), tm.st0, n * W * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(b.data(), tm.st1, n * W * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    for (int64_t i = 0; i < n; ++i) {
        float* o = us4 + 4 * i;
        o[0] = o[1] = o[2] = o[3] = -1.f;
        if (!tm.stamped[i]) continue;
        unsigned long long lo = ~0ull, hi = 0, slo = ~0ull, shi = 0, dmax = 0;
        double dsum = 0;
        int64_t nb = 0;
        for (int64_t w = 0; w < W; ++w) {
            const unsigned long long s = a[i * W + w], e = b[i * W + w];
            if (!s || e < s) continue;  // a workgroup past the stamp table, or none
            lo = std::min(lo, s);
            hi = std::max(hi, e);
            slo = std::min(slo, s);
            shi = std::max(shi, s);
            dmax = std::max(dmax, e - s);
            dsum += static_cast<double>(e - s);
            ++nb;
        }
        if (!nb) continue;
        o[0] = static_cast<float>((hi - lo) * 1e-2);  // 100 MHz ticks -> us
        o[1] = static_cast<float>(dsum / nb * 1e-2);
        o[2] = static_cast<float>(dmax * 1e-2);
        o[3] = static_cast<float>((shi - slo) * 1e-2);
    }
    return n;
}

int64_t gs_trainer_agg_times(gs_trainer* t, float* ms, int64_t cap) { return gs_trainer_kernel_times(t, 0, ms, cap); }

const char* gs_trainer_kernel_name(const gs_trainer* t, int32_t site) {
    if (!t || site < 0 || site >= gs_trainer::kSites) return "";
    return t->timer[site].kernel.c_str();
}

int gs_trainer_update_local(gs_trainer* t, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t, GS_EINVAL, "NULL argument");
    if (t->pending) {  // deferred update: the next forward (or trainer_defer_update(false)) applies it
        t->norm_ready = false;
        return GS_OK;
    }
    gs::w1_home(t, gs::as_stream(stream));  // a deferred-update step that could not defer
    const int64_t goff[3] = {0, t->cls_w_off, t->total};
    ShadowArm arm(t);
    if (t->norm_ready) {
        gs::sgd_with_parts(2, goff, t->npart, t->pstride, t->cfg.params, t->cfg.grads, t->norm_part, 1.0f,
                           t->cfg.max_norm, t->cfg.lr, gs::as_stream(stream));
    } else {
        const int rc = gs_clip_sgd(2, goff, t->cfg.params, t->cfg.grads, 1.0f, t->cfg.max_norm, t->cfg.lr,
                                   t->norm_part, stream);
        if (rc != GS_OK) return rc;
    }
    arm.done();
    t->norm_ready = false;
    GS_API_END
}

int gs_trainer_update(gs_trainer* t, float grad_scale, float* ws, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t && ws, GS_EINVAL, "NULL argument");
    t->norm_ready = false;
    GS_REQUIRE(!t->pending, GS_EINVAL, "gs_trainer_update with an update already pending");
    if (t->defer && t->defer_comm) {
        // deferred after the all-reduce: the norm partials of the summed gradient
        // and W1's speculative update in one launch; the next forward (or
        // trainer_defer_update(false)) applies the clip + SGD
        const int64_t goff[3] = {0, t->cls_w_off, t->total};
        const int64_t n1 = t->w_rows[0] * t->w_cols[0];
        const bool lowp = t->cfg.feat_dtype == GS_BF16;
        const int np = gs::sumsq_spec_launch(2, goff, t->cfg.grads, ws, t->w1_buf(t->w1_cur), t->w1_buf(t->w1_cur ^ 1),
                                             lowp ? t->lp_buf(t->w1_cur ^ 1) : nullptr, n1, t->cfg.lr, grad_scale,
                                             gs::as_stream(stream));
        t->pending = true;
        t->pend_part = ws;
        t->pend_pstride = np;
        t->pend_np[0] = np;
        t->pend_np[1] = np;
        t->pend_scale = grad_scale;
        return GS_OK;
    }
    gs::w1_home(t, gs::as_stream(stream));
    const int64_t goff[3] = {0, t->cls_w_off, t->total};
    ShadowArm arm(t);
    int rc = gs_clip_sgd(2, goff, t->cfg.params, t->cfg.grads, grad_scale, t->cfg.max_norm, t->cfg.lr, ws, stream);
    if (rc != GS_OK) return rc;
    arm.done();
    GS_API_END
}

int gs_trainer_defer(gs_trainer* t, int32_t on, int32_t* active, void* stream) {
    GS_API_BEGIN
    GS_REQUIRE(t, GS_EINVAL, "NULL argument");
    hipStream_t st = gs::as_stream(stream);
    if (active) *active = 0;
    if (on) {
        GS_REQUIRE(!t->defer && !t->pending, GS_EINVAL, "gs_trainer_defer: already deferring");
        gs::trainer_keep_lowp(t, true);  // the bf16 W1 follows every update, as in a runner loop
        const bool ok = gs::trainer_defer_update(t, true, st, true);
        if (!ok) gs::trainer_keep_lowp(t, false);
        if (active) *active = ok ? 1 : 0;
    } else {
        if (t->defer) gs::trainer_defer_update(t, false, st);
        gs::trainer_keep_lowp(t, false);
    }
    GS_API_END
}

}  // extern "C"

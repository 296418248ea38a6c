#pragma once
// Internal launchers shared between the kernel translation units and the
// trainer (step.hip).  Not part of the C-ABI: they throw gs::Error and take
// hipStream_t directly.
#include <functional>

#include "kcommon.hpp"

struct gs_trainer;
struct gs_dsampler;

namespace gs {

// step.hip: called (on the launching thread, with the step's stream) once
// every gradient except layer 1's weight gradient has been issued — after the
// layers >= 2 backward and the classifier reduce, before the layer-1 dW GEMM —
// so a caller can all-reduce the finished gradients [w1_floats, n_params)
// under that GEMM (the runner's bucketed all-reduce).  Empty: no hook.
void trainer_set_upper_hook(gs_trainer* t, std::function<void(hipStream_t)> hook);
// Layer-1 weight gradient in `chunks` row chunks (2-layer top path with an
// upper hook): after each chunk's slab sum, hook(stream, float offset into the
// gradient buffer, float count) — the runner all-reduces the chunk there, so
// only the last chunk's collective follows the step's last GEMM.  The chunks
// use the whole gradient's row slabs: the same sums bit for bit.
void trainer_set_w1_chunk_hook(gs_trainer* t, int chunks,
                               std::function<void(hipStream_t, int64_t, int64_t)> hook);
// Inside a runner loop: the SGD keeps the bf16 W1 current (no per-step cast).
void trainer_keep_lowp(gs_trainer* t, bool keep);
// Inside a runner loop without an all-reduce (fp32 2-layer steps): defer each
// step's clip + SGD into the next step's launches (gs_trainer fields defer /
// pending).  Returns whether deferral is on; off (at the end of the loop)
// applies the last pending update, so the flat parameters and gradients are
// those of the separate update launch.
bool trainer_defer_update(gs_trainer* t, bool on, hipStream_t st, bool comm = false);
int64_t trainer_w1_floats(const gs_trainer* t);

// linear.hip
// Whether gs_sage_linear_fwd takes the wide (16-B load) kernel for these
// operands: the only forward that applies a pending deferred update.
bool linear_fwd_wide_ok(gs_dtype dt, int64_t F, const void* Xs, int64_t ldxs, const void* A, int64_t lda,
                        const void* W);
int linear_dw_slabs(gs_dtype dt, int64_t n, int64_t F, int64_t H, const void* Xs, int64_t ldxs,
                    const int32_t* sidx, const void* A, int64_t lda, const float* dout, const float* out,
                    int64_t ldo, int32_t relu, float* dW, void* ws, int64_t ws_bytes, hipStream_t st,
                    int64_t H_split = -1, int phases = 1);
// Row phases of the layer-1 weight gradient (linear_dw_body<PH>): 512-thread
// workgroups, half the slabs.  Layers >= 2 keep one phase (the fused layer
// backward's slabs, which the unfused path must match).
inline constexpr int kDw1Phases = 2;
int sum_slabs_launch(const float* slabs, int S, int64_t len, float* out, float* part, hipStream_t st);
// One slab sum: out = Σ_s slabs[s] (S slabs of len floats), norm partials to part.
struct SlabSum {
    const float* slabs;
    int S;
    int64_t len;
    float* out;
    float* part;
};
// Both sums in one launch (s1 the split layer-1 sum, s2 a deferred layer-2
// sum, S2 <= 1 = nothing to add); returns s1's partial count.  s2 writes
// sum_slabs_pair_parts2(s2.len) partials.
bool sum_slabs_pair_ok(int64_t len1, int64_t len2);
int sum_slabs_pair_parts2(int64_t len2);
// spec_S: also W1's speculative update spec_S = spec_P - lr·(layer-1 sum) (the
// trainer's deferred update), and the launch takes the done flag (g_done_flag).
int sum_slabs_pair_launch(const SlabSum& s1, const SlabSum& s2, hipStream_t st, const float* spec_P = nullptr,
                          float* spec_S = nullptr, float lr = 0.f, uint16_t* spec_S_lp = nullptr);
// The pending update's tail at the end of a deferred-update run: the flat
// parameters and gradients become what the separate clip + SGD launch would
// have left (W1 from sp.S or recomputed into w1_out, the others updated).
void spec_finalize_launch(const FwdSpec& sp, float* w1_out, int64_t w1_floats, hipStream_t st);
int sum_slabs_grid(int64_t len);

// agg.hip: the runner's layer-1 gather in two launches (resolve, then rows)
void resolve_ids_launch(int64_t n_dst, int k, const int32_t* ptr, const int32_t* ent, const int32_t* col,
                        const int32_t* dst_ids, int gcn, int32_t* ids, hipStream_t st);
// resolve_ids_launch plus the fused top launch's padded hop-1 records
// (tout[r][0] = self, [1..tk] = the list, -1 past it; n_top roots) and, with
// n_rec > 0, the layer-2 backward's per-row records of the transposed hop-1
// lists (rout[c] = {n, beg, e0 .. e5}, agg_bwd_rec_body; n_rec = |L1|).
void resolve_top_launch(int64_t n_dst, int k, const int32_t* ptr, const int32_t* ent, const int32_t* col,
                        const int32_t* dst_ids, int gcn, int32_t* ids, int64_t n_top, int tk, const int32_t* tptr,
                        const int32_t* tnbr, const int32_t* tself, int32_t* tout, hipStream_t st, int64_t n_rec = 0,
                        const int32_t* rptr = nullptr, const int32_t* ridx = nullptr, int32_t* rout = nullptr);
// Padded hop-1 records for the fused top launch, one buffer per gather slot
// (2-layer training steps; B roots, fanout tk <= 31).
void trainer_reserve_top(gs_trainer* t, int64_t B, int32_t tk);
// self_out (optional): each destination's own row X[dst_ids[r]] copied to self_out[r]
void agg_ids_launch(gs_agg op, gs_dtype dt, const void* X, int64_t ldx, int64_t F, int64_t n_dst, int k,
                    const int32_t* ids, const int32_t* dst_ids, int gcn, void* out, int64_t ldo, hipStream_t st,
                    void* self_out = nullptr, int64_t ldso = 0);

// misc.hip
int cls_rows_launch(int64_t B, int64_t D, int64_t C, const float* E, const float* Wc, const float* bc,
                    const int32_t* labels, const int32_t* roots, int32_t mask_relu, float* dE, float* ws,
                    hipStream_t st);
void sgd_with_parts(int32_t n_groups, const int64_t* goff_host, const int* npart, int pstride, float* params,
                    float* grads, const float* part, float grad_scale, float max_norm, float lr, hipStream_t st);
// The deferred update after an all-reduce: gs_clip_sgd's norm partials (into
// part, kNormBlocks per group; returns that count) and W1's speculative update
// S = P - lr·(scale·g) (+ S_lp in bf16) for the elements [0, n1); takes the
// done flag.
int sumsq_spec_launch(int32_t n_groups, const int64_t* goff_host, const float* grads, float* part, const float* P,
                      float* S, uint16_t* S_lp, int64_t n1, float lr, float scale, hipStream_t st);

// bwd.hip: the backward of one layer l >= 2 (fp32 activations, relu already
// folded into dZ) in two launches, each running independent kernels side by
// side in one grid (every boundary between dependent launches costs the
// stream a drain and a dispatch, ~2-3 us measured):
//   A: dW_l row slabs | dIn_l = dZ_l · W_l | (top layer) classifier reduce
//   B: dW_l = Σ slabs (+ its norm partials) | agg backward into dH_{l-1}
struct LayerBwd {
    int64_t n, fin, H;                    // rows, input width per concat half, output width
    const float* Xs;                      // self rows source (nullptr: gcn), row stride ldxs
    int64_t ldxs;
    const int32_t* sidx;                  // self row of each output row
    const float* A;                       // aggregate [n][fin], row stride lda (0: fin)
    int64_t lda = 0;
    const float* dZ;                      // [n][H], already masked by relu'
    const float* W;                       // [H][K]
    float* dW;                            // [H][K] gradient
    float* slabs;                         // dW row slabs workspace
    int64_t slab_bytes;
    float* dIn;                           // [n][K] input gradient ([dSelf | dA], or dA when gcn)
    int agg;                              // GS_AGG_MEAN / GS_AGG_MAX
    int64_t n_src;                        // rows of the previous layer
    const int32_t* tptr;                  // transposed neighbourhoods (GS_PK_TPTR / TIDX)
    const int32_t* tidx;
    const int32_t* ptr;                   // forward neighbourhood offsets (mean weights)
    const int32_t* argmax;                // MAX routing, [n][H]
    const int4* trec = nullptr;           // optional per-source records (agg_bwd_rec_body), n_src rows
    const float* Hprev;                   // previous layer's output (relu mask), [n_src][H]
    float* dH;                            // [n_src][H] gradient of the previous layer's output (masked)
    bool din_ready = false;               // dIn already written (top.hip): launch A skips its dIn role
    int64_t din_off2 = 0;                 // dIn as two partials, the second din_off2 floats on (the top pair form)
};

struct ClsReduce {
    int64_t B, D, C;
    int n_row_blocks;
    const float* slab;
    float* dWc;
    float* dbc;
    float* loss;
    float* part;                          // norm partials of (dWc, dbc), one per reduce block
};
// The fused top path's one backward launch for layer 2 (bwd.hip): dW_2 slabs,
// classifier reduce and the agg backward to dH_1; the dW_2 slab sum is left
// in *deferred (S <= 1: dW_2 written directly) for sum_slabs_pair_launch.
// Returns the norm partials that sum will write (placed first, as layer_bwd's).
// Roles of the fused layer-2 backward launches (bwd.hip).
struct BwdA {
    int n, F, H, K, rps;
    const float* Xs;
    int64_t ldxs;
    const int* sidx;
    const float* A;
    int64_t lda;    // A's row stride (F, or 2F for the top path's dense [self | agg] rows)
    const float* dZ;
    float* target;  // dW slabs (or dW itself when S == 1)
    int dw_gx, dw_gy, dw_nb;
    const float* W;
    float* dSelf;
    float* dA;
    int dx_gx, dx_nb;
    // classifier reduce (top layer only)
    int B, D, C, cls_rows;
    const float* cls_slab;
    float* dWc;
    float* dbc;
    float* loss;
    float* cls_part;
};
int layer_bwd_top(const LayerBwd& a, const ClsReduce& cls, SlabSum* deferred, hipStream_t st);

bool layer_bwd_fusable(const LayerBwd& a);
int cls_reduce_grid(int64_t C, int64_t D);
// Returns the number of norm partials written to `part` (0 when the weight
// gradient fits one slab and was written directly: no partials).
int layer_bwd(const LayerBwd& a, const ClsReduce* cls, float* part, hipStream_t st);

// top.hip: a 2-layer model's layer 2 forward (aggregate + linear + relu), the
// loss head and the layer's dIn in one launch (one block per 4 roots).
// aggo receives each root's dense [self | agg] input row (2H floats: the
// layer-2 weight gradient then reads no self index).
// Returns the number of classifier partial slabs written (the loss head's).
bool top_supported(int64_t H, int64_t C, bool gcn);
// tids: optional padded hop-1 records (resolve_top_launch, 1 + tk ids per
// root); nullptr reads the pack's lists (ptr, nbr, self).
int top_fwd_bwd(int agg, int64_t B, int64_t C, const float* Hprev, const int32_t* ptr, const int32_t* nbr,
                const int32_t* self, const float* W, const float* Wc, const float* bc, const int32_t* labels,
                const int32_t* roots, float* aggo, int32_t* argmax, float* E, float* dZ, float* dIn, float* slab,
                hipStream_t st, const int32_t* tids = nullptr, int tk = 0);
// The pair form (C <= 16): two blocks per 4 roots, each with half of W2 and
// E's columns, the partial logits exchanged between the pair as tagged
// granules (xch: [8·ceil(quads / 8)][2][64] u64, zero at allocation; epoch:
// the launch's tag, never 0 and never repeated on one buffer; fail: set if a
// block gave up waiting, its outputs are then NaN).  dIn receives half 0's
// partial of the input gradient, dIn2 half 1's: the consumer adds them,
// dIn + dIn2 (LayerBwd::din_off2).  Returns the classifier slabs written.
bool top_pair_supported(int64_t H, int64_t C, bool gcn);
int top_pair_fwd_bwd(int agg, int64_t B, int64_t C, const float* Hprev, const int32_t* ptr, const int32_t* nbr,
                     const int32_t* self, const float* W, const float* Wc, const float* bc, const int32_t* labels,
                     const int32_t* roots, float* aggo, int32_t* argmax, float* E, float* dZ, float* dIn, float* dIn2,
                     float* slab, unsigned long long* xch, unsigned epoch, unsigned* fail, hipStream_t st,
                     const int32_t* tids = nullptr, int tk = 0);
inline int64_t top_pair_xch_words(int64_t B) { return 8 * ((((B + 3) / 4) + 7) / 8) * 2 * 64; }

// dsample.hip: whether the last gs_dsampler_run has completed (no wait).
bool dsampler_ready(gs_dsampler* ds);
bool dsampler_run_ready(gs_dsampler* ds, int64_t run);  // run number `run` has finished

}  // namespace gs

/*
 * graphsage_amd.h — C-ABI of libgraphsage_amd.so, the MI355X-native GraphSAGE
 * sample-and-aggregate path.
 *
 * Plain C types only: pointers, sizes, enums.  No torch types cross this line.
 * Every function returns an int status (GS_OK == 0); on failure the calling
 * thread's message is available from gs_last_error().  Device entry points are
 * asynchronous on the caller's hipStream_t (passed as void*) and never allocate
 * or synchronise: the caller owns every buffer (the Python host allocates them
 * through the torch caching allocator).
 *
 * Each entry point names the reference code it stands in for
 * (paths relative to Lolash/graphSAGE-pytorch).
 */
#ifndef GRAPHSAGE_AMD_H
#define GRAPHSAGE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
#define GS_OK 0
#define GS_EINVAL 1  /* bad argument (ValueError in the Python host)              */
#define GS_ENOMEM 2  /* host allocation failed                                    */
#define GS_EHIP 3    /* HIP runtime error (launch/config)                         */
#define GS_ERANGE 4  /* "Sample larger than population" / id out of range          */
#define GS_EEMPTY 5  /* MAX over an empty neighbourhood (reference: IndexError,
                        models.py:321-325)                                       */
#define GS_ELIMIT 6  /* a device-path capacity was exceeded (device sampler: a
                        rejection window, walk or frontier table too small for
                        this batch); the host path computes the same result, and
                        the stream state the caller holds is untouched            */

const char* gs_last_error(void);
const char* gs_version(void);

/* ------------------------------------------------------------------- RNG
 * CPython 3.10 `random.Random` (MT19937) stream.  The reference draws every
 * neighbour sample from the module-global `random` (models.py:281-282) and
 * shares that stream with UnsupervisedLoss (models.py:164,178); the handle
 * below is interchangeable with random.getstate()/setstate() (version 3). */
typedef struct gs_rng gs_rng;

int gs_rng_create(gs_rng** out);
void gs_rng_destroy(gs_rng* rng);
/* random.seed(n) for an int n: key = little-endian 32-bit words of abs(n)
 * (main.py:40 seeds with 824). */
int gs_rng_seed_words(gs_rng* rng, const uint32_t* key, int64_t key_len);
/* random.setstate((3, mt[0..623] + (pos,), gauss)) / getstate(). */
int gs_rng_set_state(gs_rng* rng, const uint32_t* mt624, int64_t pos);
int gs_rng_get_state(const gs_rng* rng, uint32_t* mt624, int64_t* pos);
/* Known-answer helpers: getrandbits(k) (k<=32) and _randbelow(n), `count` times. */
int gs_rng_getrandbits(gs_rng* rng, int32_t k, int64_t count, uint32_t* out);
int gs_rng_randbelow(gs_rng* rng, uint32_t n, int64_t count, uint32_t* out);
/* random.sample(range(n), k) as positions (both CPython branches, random.py
 * sample(); what models.py:282 calls on tuple(adj_set)). */
int gs_rng_sample_positions(gs_rng* rng, int64_t n, int64_t k, int64_t* out);
/* random.choice(seq) position for len(seq)==n (models.py:178). */
int gs_rng_choice_position(gs_rng* rng, int64_t n, int64_t* out);

/* ------------------------------------------------- CPython set known answers
 * list(set.union(*[set(l) for l in lists])) — the set(list) + union that
 * produce the frontier order at models.py:282-286.  out must hold Σ len. */
int gs_pyset_union_of_lists(const int64_t* items, const int64_t* ptr,
                            int64_t n_lists, int64_t* out, int64_t* out_len);

/* ------------------------------------------------------------------ graph
 * Adjacency in CPython-set iteration order.  Replaces the dict-of-sets built
 * by DataCenter (dataCenter.py:33-41 cora, :77-86 pubmed):
 *   for (a, b) in pairs: adj[a].add(b); adj[b].add(a)
 * Row v of the CSR lists tuple(adj[v]) — the population random.sample sees.
 * The slot layout of each row's set is kept (host side) because a row with
 * fewer than k neighbours enters the frontier union as that very set
 * (models.py:282, :285). */
typedef struct gs_graph gs_graph;

int gs_graph_build(const int64_t* src, const int64_t* dst, int64_t n_pairs,
                   int64_t n_nodes, int32_t n_threads, gs_graph** out);
/* Adopt rows whose set layout the caller read from live CPython set objects
 * (the drop-in path: GraphSage(adj_lists=...) with a caller-built dict of
 * sets).  Per row v: entries row_ptr[v]..row_ptr[v+1] in slot order, slot[e]
 * their table slots (strictly increasing), table size 1 << log2size[v];
 * dirty[v] != 0 when the set holds dummy entries (fill != used).  dirty may
 * be NULL. */
int gs_graph_from_tables(int64_t n_nodes, const int64_t* row_ptr,
                         const int32_t* col, const uint32_t* slot,
                         const uint8_t* log2size, const uint8_t* dirty,
                         gs_graph** out);
void gs_graph_destroy(gs_graph* g);
int gs_graph_dims(const gs_graph* g, int64_t* n_nodes, int64_t* n_entries,
                  int64_t* max_degree);
/* Borrowed views, valid until gs_graph_destroy: row_ptr[n_nodes+1], col[n_entries]. */
const int64_t* gs_graph_row_ptr(const gs_graph* g);
const int32_t* gs_graph_col(const gs_graph* g);
/* One node-wide CSR shared by the rank processes (the replicated
 * adjacency of dataCenter.py:33-41, built once per node).  A flat image —
 * header, row_ptr, col, slot, log2size, dirty, 64-byte aligned — that local
 * rank 0 writes (to a /dev/shm file) and every rank maps read-only and adopts
 * without a copy.  gs_graph_from_image keeps pointers into `img`: the caller
 * keeps it mapped until gs_graph_destroy.  The sampler reads an adopted graph
 * exactly as one it built itself. */
int64_t gs_graph_image_bytes(const gs_graph* g);
int gs_graph_write_image(const gs_graph* g, void* dst, int64_t cap);
int gs_graph_from_image(const void* img, int64_t bytes, gs_graph** out);

/* Synthetic R-MAT(a,b,c,1-a-b-c) pair list: `scale` id bits,
 * n_pairs draws, self pairs dropped, optional seeded id permutation.
 * src/dst must hold n_pairs; *n_kept receives the pairs written. */
int gs_rmat_pairs(int32_t scale, int64_t n_pairs, double a, double b, double c,
                  uint64_t seed, int32_t permute, int32_t n_threads,
                  int64_t* src, int64_t* dst, int64_t* n_kept);

/* ---------------------------------------------------------------- sampler
 * GraphSage._get_unique_neighs_list (models.py:277-289) for every hop of a
 * forward (models.py:246-251), consuming the rng exactly as the reference.
 *
 * Hops are numbered from the roots: hop 1 samples the roots (frontier F0 =
 * nodes_batch) and its union is F1; hop j samples F(j-1) and unions into Fj.
 * fanouts[j-1] = num_sample of hop j (the reference hard-codes 10); <=0 means
 * "no sampling" (num_sample=None, models.py:283-284).
 *
 * The last hop's union (the deepest frontier, L0 of the reference) only feeds
 * a row gather, so unless GS_SAMPLE_FULL is set it is not materialised: its
 * sampled *positions* go to the device, which expands them through the CSR. */
#define GS_SAMPLE_GCN 1  /* gcn=True: self stays in its own neighbourhood      */
#define GS_SAMPLE_FULL 2 /* materialise the last hop's sets + union (API/parity) */
#define GS_MAX_HOPS 8

typedef struct gs_sample gs_sample;

typedef struct {
    int64_t n_dst;            /* |F(j-1)|                                       */
    int64_t n_pos;            /* sampled row positions = Σ min(deg, k)           */
    int64_t n_src;            /* |Fj|, -1 when not materialised                  */
    int64_t n_nbr;            /* neighbourhood entries after the self rule, -1   */
    const int64_t* dst_ids;   /* [n_dst] F(j-1) in order                         */
    const int32_t* pos_ptr;   /* [n_dst+1]                                       */
    const int32_t* pos;       /* [n_pos] positions into CSR row of dst, in
                                 random.sample result order (or row order)       */
    const int64_t* src_ids;   /* [n_src] Fj in CPython set order (models.py:286) */
    const int32_t* nbr_ptr;   /* [n_dst+1]                                       */
    const int32_t* nbr;       /* [n_nbr] index into src_ids, ascending per dst
                                 (the dense mask's column order, models.py:306)  */
    const int32_t* self_local;/* [n_dst] index of dst in Fj (_nodes_map :271)    */
    const int32_t* set_ptr;   /* [n_dst+1] samp_neighs[i] incl. self, iteration */
    const int64_t* set_items; /*   order of the reference's set object           */
    int64_t n_empty;          /* destinations with no neighbour after the self
                                 rule (MEAN gives NaN, MAX raises IndexError)    */
} gs_hop_view;

/* Device pack: everything the kernels read for one batch, one int32 buffer. */
enum {
    GS_PK_POS_PTR = 0, /* last hop: [n_dst+1]                                 */
    GS_PK_POS,         /* last hop: [n_pos] absolute CSR entries
                          row_ptr[dst] + position (the hop view's pos + row
                          start), so the device gather skips row_ptr      */
    GS_PK_DST_IDS,     /* last hop: [n_dst] global ids of F(L-1)              */
    GS_PK_NBR_PTR,     /* hops < L: [n_dst+1]                                 */
    GS_PK_NBR,         /* hops < L: [n_nbr]                                   */
    GS_PK_SELF,        /* hops < L: [n_dst]                                   */
    GS_PK_TPTR,        /* hops < L: transposed CSR over Fj, [n_src+1]         */
    GS_PK_TIDX,        /* hops < L: [n_nbr + n_dst] per source c, ascending r:
                          r >= 0 → c is in dst r's neighbourhood,
                          -(r+1) → c is dst r's own (self) row               */
    GS_PK_NFIELDS
};

typedef struct {
    int64_t total;                               /* int32 elements            */
    int64_t off[GS_MAX_HOPS][GS_PK_NFIELDS];     /* element offsets, -1 absent */
} gs_pack_layout;

int gs_sample_run(const gs_graph* g, gs_rng* rng, const int64_t* roots,
                  int64_t n_roots, const int32_t* fanouts, int32_t n_hops,
                  int32_t flags, gs_sample** out);
void gs_sample_destroy(gs_sample* s);
int gs_sample_n_hops(const gs_sample* s, int32_t* n_hops);
int gs_sample_hop(const gs_sample* s, int32_t hop, gs_hop_view* out);
int gs_sample_pack_layout(const gs_sample* s, gs_pack_layout* out);
/* Writes the layout's int32 image into buf (cap elements, typically pinned). */
int gs_sample_pack(const gs_sample* s, int32_t* buf, int64_t cap);

/* Streaming form for sampler threads: sample every hop and write the device
 * image plus the roots (int32, at element `used - n_roots`) straight into a
 * caller buffer of at least gs_sample_pack_bound() elements, with no handle
 * to keep.  hop_sizes[4*j..] = (n_dst, n_pos, n_src, n_nbr) of hop j+1;
 * offsets = gs_pack_layout.off flattened.  GS_SAMPLE_FAIL_EMPTY turns an
 * empty neighbourhood into GS_EEMPTY (MAX aggregation). */
#define GS_SAMPLE_FAIL_EMPTY 4
int64_t gs_sample_pack_bound(const gs_graph* g, int64_t n_roots,
                             const int32_t* fanouts, int32_t n_hops);
int gs_sample_pack_run(const gs_graph* g, gs_rng* rng, const int64_t* roots,
                       int64_t n_roots, const int32_t* fanouts, int32_t n_hops,
                       int32_t flags, int32_t* buf, int64_t cap,
                       int64_t* hop_sizes, int64_t* offsets, int64_t* used);
/* Several batches in one pack (the inference runner's merged launches): the
 * roots split into consecutive groups of `group` ids (the last one may be
 * shorter), each group sampled on its own, in order, from `rng` — exactly
 * the draws of one gs_sample_pack_run per group — and the groups' images
 * concatenated field by field with their indices rebased, so each row's
 * neighbourhood and every kernel's result for it are those of its own batch.
 * hop_sizes are the groups' sums.  n_roots <= group: gs_sample_pack_run. */
int64_t gs_sample_pack_bound_multi(const gs_graph* g, int64_t n_roots, int64_t group,
                                   const int32_t* fanouts, int32_t n_hops);
int gs_sample_pack_run_multi(const gs_graph* g, gs_rng* rng, const int64_t* roots,
                             int64_t n_roots, int64_t group, const int32_t* fanouts,
                             int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap,
                             int64_t* hop_sizes, int64_t* offsets, int64_t* used);
/* Helper threads for one sampling stream (not a reference interface: they
 * split the RNG-independent parts of a batch — the per-node set builds of
 * models.py:282-285 and the neighbour / transposed lists a hop's aggregate
 * needs — while the calling thread keeps the sequential draws and union).
 * The result is bit-identical to the team-less call.  A team serves one
 * calling thread at a time. */
typedef struct gs_team gs_team;
int gs_team_create(int32_t helpers, gs_team** out);
/* A second handle on peer's helper threads (one pool for several sampling
 * streams: a stream's set builds take whatever helpers the others leave
 * idle).  Each handle still serves one calling thread; the threads live
 * until the last handle on them is destroyed. */
int gs_team_create_shared(const gs_team* peer, gs_team** out);
void gs_team_destroy(gs_team* team);
/* gs_sample_pack_run_multi with a team (NULL: none). */
int gs_sample_pack_run_multi_team(const gs_graph* g, gs_rng* rng, const int64_t* roots,
                                  int64_t n_roots, int64_t group, const int32_t* fanouts,
                                  int32_t n_hops, int32_t flags, int32_t* buf, int64_t cap,
                                  int64_t* hop_sizes, int64_t* offsets, int64_t* used,
                                  gs_team* team);

/* ------------------------------------------------------- device sampler
 * The same sampling as gs_sample_pack_run (models.py:246-251 over
 * _get_unique_neighs_list, models.py:277-289), run on the GPU from a device
 * copy of the graph and a device MT19937 stream: the pack lands in device
 * memory, bit-identical to the host sampler's image, and the stream advances
 * exactly as the reference's `random` would.  One handle is one
 * stream; its calls are ordered on the caller's stream.  Fanouts <= 32. */
typedef struct gs_dsampler gs_dsampler;
/* gs_dsampler_create flag: every kernel on the caller's stream.  By default a
 * sampler owns an aux stream that runs the union lists of the hop before the
 * last and the next run's MT19937 words beside the last hop's draws (one
 * fork, one join per run) — it pays for one sampler alone on the GPU, not for
 * several sharing it (the runner sets this flag for S > 1). */
#define GS_DSAMPLER_NO_AUX 8
int gs_dsampler_create(const gs_graph* g, const int32_t* fanouts, int32_t n_hops,
                       int64_t max_roots, int32_t flags, gs_dsampler** out);
void gs_dsampler_destroy(gs_dsampler* ds);
/* random.setstate / getstate on the device stream (both synchronise). */
int gs_dsampler_set_rng(gs_dsampler* ds, const uint32_t* mt624, int64_t pos, void* stream);
int gs_dsampler_get_rng(gs_dsampler* ds, uint32_t* mt624, int64_t* pos, void* stream);
/* Known answers: the next n words of the stream (genrand_uint32 outputs),
 * without consuming them (synchronises). */
int gs_dsampler_words(gs_dsampler* ds, int64_t n, uint32_t* out, void* stream);
/* Elements a pack of n_roots roots may need (gs_sample_pack_bound + roots). */
int64_t gs_dsampler_pack_bound(const gs_dsampler* ds, int64_t n_roots);
/* Sample one batch (device int32 roots) into a device pack, asynchronously on
 * `stream`; gs_dsampler_result waits for it and reports the layout exactly as
 * gs_sample_pack_run does (hop_sizes, offsets, used), or its error. */
int gs_dsampler_run(gs_dsampler* ds, const int32_t* roots, int64_t n_roots, int32_t* pack,
                    int64_t cap, void* stream);
int gs_dsampler_result(gs_dsampler* ds, int64_t* hop_sizes, int64_t* offsets, int64_t* used);
/* Runs issued so far on this sampler; run i (0-based) is gs_dsampler_run's
 * i-th call.  gs_dsampler_result_of(ds, i, ...) reports run i's layout (waits
 * for that run only), so a caller may keep a second run queued behind the one
 * it reads; the last 4 runs are kept (GS_ERANGE for older ones). */
int64_t gs_dsampler_runs(const gs_dsampler* ds);
int gs_dsampler_result_of(gs_dsampler* ds, int64_t run, int64_t* hop_sizes, int64_t* offsets, int64_t* used);
/* Diagnostics of the last run (waits for it): n <= 64 words — per-phase
 * device timestamps (100 MHz) and round counts of the frontier union's
 * stages; the layout is documented in kernels/dsample_union.hip. */
int gs_dsampler_debug(gs_dsampler* ds, int64_t* out, int32_t n);

/* ------------------------------------------------- unsupervised-loss batch
 * UnsupervisedLoss (models.py:30-186) over the same graph and rng:
 * extend_nodes (models.py:135-147, called by apply_model at utils.py:149)
 * consumes the stream exactly as the reference — random walks
 * (random.choice, models.py:178) in node order, then per node the
 * n_walk_len-hop ball and random.sample(set(train) - ball, num_neg)
 * (models.py:152-164) — and returns list(set(pos) | set(neg))
 * (models.py:146) in CPython set order.  Balls are grown on n_threads
 * threads; the draws stay in node order.  Reference constants: n_walks 6,
 * walk_len 1, n_walk_len 5 (models.py:36-39). */
typedef struct gs_unsup gs_unsup;

int gs_unsup_create(const gs_graph* g, const int64_t* train_nodes, int64_t n_train,
                    int32_t n_walks, int32_t walk_len, int32_t n_walk_len,
                    gs_unsup** out);
void gs_unsup_destroy(gs_unsup* u);
/* Grow the n_walk_len-hop balls (models.py:154-162) on the GPU — a
 * bit-parallel multi-source BFS, 64 balls per 64-bit word — and pick the
 * negatives' far-list elements there (select queries over set(train)'s order
 * with the ball's members skipped); the draws of models.py:164 stay on the
 * calling thread in node order, so every result and the rng stream are those
 * of the host path.  Uploads the CSR once to the current
 * device.  The device half owns a non-blocking stream there (each extend
 * synchronises only that stream); `stream` is unused and may be NULL. */
int gs_unsup_attach_device(gs_unsup* u, void* stream);
/* parts: 1 = the walks only (get_positive_nodes, models.py:149), 2 = the
 * negatives only (get_negtive_nodes, :152), 3 = both (extend_nodes).
 * sizes[4] = (len(unique_nodes_batch), len(positive_pairs),
 * len(negtive_pairs), set(nodes) < set(unique) ? 1 : 0 — the assertion at
 * models.py:147, which the Python host raises). */
int gs_unsup_extend(gs_unsup* u, gs_rng* rng, const int64_t* nodes, int64_t n,
                    int64_t num_neg, int32_t parts, int32_t n_threads,
                    int64_t* sizes);
/* Copy out the last extend: unique[sizes0], pos_pairs[2*sizes1] and
 * neg_pairs[2*sizes2] as (node, other) in append order, per input node its
 * positive / negative pair counts and has_pos (node is a key of
 * node_positive_pairs, i.e. its adjacency set is non-empty).  NULL skips. */
int gs_unsup_fetch(const gs_unsup* u, int64_t* unique, int64_t* pos_pairs,
                   int64_t* neg_pairs, int64_t* pos_cnt, int64_t* neg_cnt,
                   uint8_t* has_pos);
/* Index plan of get_loss_sage / get_loss_margin (models.py:65-132) for the
 * last extend, int32, rows = positions in unique (node2index, :69):
 *   pos_ptr[M+1] | neg_ptr[M+1] | pos_a[P] | pos_b[P] | neg_a[N] | neg_b[N]
 *   | tptr[U+1] | tidx[2(P+N)]
 * M scored nodes (both pair lists non-empty, dict order), tidx = 2*pair +
 * side per embedding row, ascending.  dims[6] = (M, P, N, U,
 * len(node_positive_pairs), len(node_negtive_pairs)); *used = elements.
 * buf == NULL only reports dims / used. */
int gs_unsup_loss_plan(const gs_unsup* u, int32_t* buf, int64_t cap,
                       int64_t* dims, int64_t* used);

/* --------------------------------------------------------- device kernels */
typedef enum { GS_F32 = 0, GS_BF16 = 1 } gs_dtype;
typedef enum { GS_AGG_MEAN = 0, GS_AGG_MAX = 1 } gs_agg;

/* Fill X[N, F] (row stride ld) with U(-1,1) from a counter hash of
 * (seed, row, col) — the synthetic feature table. */
int gs_fill_uniform(void* X, gs_dtype dt, int64_t N, int64_t F, int64_t ld,
                    uint64_t seed, void* stream);
/* Mirror of the host feature hash for checks (fp32, n values). */
int gs_uniform_host(uint64_t seed, int64_t row0, int64_t F, int64_t n_rows,
                    float* out);

/* GraphSage.aggregate (models.py:291-330): mean (mask/rowsum @ X, :311-314)
 * or element-wise max (:316-326) of source rows per destination.
 *   explicit mode (col == NULL): sources of dst r are rows idx[ptr[r]..ptr[r+1]).
 *   expand mode (col != NULL): node = dst_ids[r]; sources are
 *     col[row_ptr[node] + idx[e]] (positions), or col[idx[e]] when row_ptr is
 *     NULL (absolute CSR entries, as gs_sample_pack writes them), minus node
 *     itself unless gcn; gcn adds node once (models.py:285, :297-298).
 * MEAN of an empty neighbourhood is NaN like the reference (0/0); MAX of one
 * is reported as GS_EEMPTY by the host before launch.  argmax (MAX, optional)
 * receives the winning source row per element, first index on ties. */
int gs_agg_fwd(gs_agg op, gs_dtype xdt, const void* X, int64_t ldx, int64_t F,
               int64_t n_dst, const int32_t* ptr, const int32_t* idx,
               const int64_t* row_ptr, const int32_t* col,
               const int32_t* dst_ids, int32_t gcn,
               void* out, gs_dtype odt, int64_t ldo, int32_t* argmax,
               void* stream);

/* SageLayer.forward (models.py:209-220):
 *   out[n, H] = relu( [Xs[sidx[i]] | A[i]] · Wᵀ )   (cat order self first, :216)
 * Xs == NULL → gcn form out = relu(A · Wᵀ) with W [H, F] (:218).
 * sidx == NULL → identity.  W is [H, K] with K = 2F (or F); Wd is W in the
 * compute dtype (== W for GS_F32).  Inputs of dtype dt, fp32 accumulate. */
int gs_sage_linear_fwd(gs_dtype dt, int64_t n, int64_t F, int64_t H,
                       const void* Xs, int64_t ldxs, const int32_t* sidx,
                       const void* A, int64_t lda, const void* Wd,
                       float* out, int64_t ldo, int32_t relu, void* stream);

/* Autograd of SageLayer (utils.py:184 through models.py:219):
 *   dZ = dOut ⊙ (out > 0)        (relu backward; relu=0 → dZ = dOut)
 *   dW[H, K] = dZᵀ · [Xs[sidx] | A]      (overwritten)
 * ws: fp32 workspace of gs_sage_linear_bwd_weight_ws(n, K, H) bytes. */
int64_t gs_sage_linear_bwd_weight_ws(int64_t n, int64_t K, int64_t H);
int gs_sage_linear_bwd_weight(gs_dtype dt, int64_t n, int64_t F, int64_t H,
                              const void* Xs, int64_t ldxs, const int32_t* sidx,
                              const void* A, int64_t lda,
                              const float* dout, const float* out, int64_t ldo,
                              int32_t relu, float* dW, void* ws, int64_t ws_bytes,
                              void* stream);
/*   dIn[n, K] = dZ · W, written as dSelf[n, F] | dA[n, F] (dSelf NULL in gcn). */
int gs_sage_linear_bwd_input(int64_t n, int64_t F, int64_t H,
                             const float* dout, const float* out, int64_t ldo,
                             int32_t relu, const float* W,
                             float* dSelf, float* dA, int64_t ldd, void* stream);

/* Backward of aggregate + the self-row gather of the next layer
 * (models.py:265 `pre_hidden_embs[nb]`, :314 mask.mm), over source rows c of
 * the previous hidden state, with the transposed CSR of one hop
 * (GS_PK_TPTR / GS_PK_TIDX encoding):
 *   g[c] = Σ_{t ∈ tptr[c]..tptr[c+1]}  tidx[t] = -(r+1) : dSelf[r]
 *                          (skipped when dSelf == NULL: gcn mode)
 *                                       tidx[t] = r      : MEAN dA[r] / deg(r)
 *                                                          MAX  dA[r] where argmax[r] == c
 *   dH[c] = g[c] ⊙ (Hprev[c] > 0)   (the relu of the layer below; Hprev NULL → g)
 * deg(r) = ptr[r+1] - ptr[r] of the forward neighbourhood.  Deterministic:
 * no atomics, fixed summation order. */
int gs_agg_bwd(gs_agg op, int64_t n_src, int64_t F, const int32_t* tptr,
               const int32_t* tidx, const int32_t* ptr,
               const float* dA, const float* dSelf, int64_t ldd,
               const int32_t* argmax, const float* Hprev, int64_t ldh,
               float* dH, void* stream);

/* Layer 1 of GraphSage.forward (models.py:255-260) fused: the expand-mode
 * gather-aggregate of gs_agg_fwd (absolute CSR entries `ent`, self dropped
 * unless gcn) feeding gs_sage_linear_fwd's relu([X[dst] | agg] · Wᵀ) through
 * LDS, in one launch.  Writes the aggregate rows to agg_out (dtype dt, kept
 * for the weight gradient) and out[n_dst, H] (fp32).  Results equal the
 * two-kernel path bitwise.  col == NULL selects explicit mode (layers >= 2):
 * ent holds the source rows of X themselves (the pack's NBR lists, already
 * self-filtered) and dst_ids the self rows (SELF field), like gs_agg_fwd's
 * explicit mode.  gs_sage1_fwd_supported: 1 when the 16-row A tile
 * fits 64 KiB of LDS (F <= 512 fp32 / 1024 bf16 with self) and F is a
 * multiple of the 16-byte vector. */
int gs_sage1_fwd_supported(gs_dtype dt, int64_t F, int64_t H, int32_t gcn);
int gs_sage1_fwd(gs_agg op, gs_dtype dt, const void* X, int64_t ldx, int64_t F,
                 int64_t H, int64_t n_dst, const int32_t* ptr, const int32_t* ent,
                 const int32_t* col, const int32_t* dst_ids, int32_t gcn,
                 const void* W, void* agg_out, int64_t ld_agg, float* out,
                 int64_t ldo, int32_t relu, void* stream);

/* Classification (models.py:8-27) + NLL mean (utils.py:159-164), fused
 * forward + backward: logits = E·Wcᵀ + bc, logp = log_softmax (max-shifted),
 * loss = -Σ_i logp[i, y_i] / B with y_i = labels[roots[i]] (labels[i] when
 * roots is NULL, utils.py:161); writes loss[0], dE[B,D], dWc[C,D], dbc[C]
 * (all overwritten).  mask_relu != 0 zeroes dE where E <= 0 (E = relu output
 * of the last SageLayer, so dE is that layer's dZ).  C + D < 16384.
 * ws: gs_cls_nll_ws_floats(B, D, C) floats.  Deterministic (fixed-order
 * partial sums, no atomics); two launches. */
int64_t gs_cls_nll_ws_floats(int64_t B, int64_t D, int64_t C);
int gs_cls_nll_fwd_bwd(int64_t B, int64_t D, int64_t C, const float* E,
                       const float* Wc, const float* bc, const int32_t* labels,
                       const int32_t* roots, int32_t mask_relu, float* loss,
                       float* dE, float* dWc, float* dbc, float* ws,
                       void* stream);

/* get_loss_sage (kind 0, models.py:65-96) / get_loss_margin (kind 1,
 * models.py:98-132) over a device copy of gs_unsup_loss_plan:
 *   sage  : mean_m [ -mean_p log σ(cos⁺) - q · mean_n log σ(-cos⁻) ]
 *   margin: mean_m max(0, max_n log σ(cos⁻) - min_p log σ(cos⁺) + margin)
 * with cos = F.cosine_similarity (eps 1e-8) of embedding rows emb[U, D]
 * (D % 4 == 0, <= 1024, 16-byte aligned rows).  The forward (two launches)
 * writes loss[0] and keeps per-pair state in ws
 * (gs_unsup_loss_ws_floats floats, 16-byte aligned); the backward (one
 * launch) writes dE[U, D] = dloss[0] · ∂loss/∂emb, every row overwritten,
 * in a fixed summation order (no atomics).  Reference constants: q = 10,
 * margin = 3 (models.py:35, :40). */
int64_t gs_unsup_loss_ws_floats(int64_t M, int64_t P, int64_t N);
int gs_unsup_loss_fwd(int32_t kind, int64_t M, int64_t P, int64_t N, int64_t U,
                      int64_t D, const float* emb, int64_t lde, const int32_t* plan,
                      float q, float margin, float* loss, float* ws, void* stream);
int gs_unsup_loss_bwd(int64_t M, int64_t P, int64_t N, int64_t U, int64_t D,
                      const float* emb, int64_t lde, const int32_t* plan,
                      const float* ws, const float* dloss, float* dE, int64_t ldd,
                      void* stream);

/* clip_grad_norm_(params, max_norm) per group (utils.py:185-186) then SGD
 * (utils.py:136,187): p -= lr * g * min(1, max_norm / (||g_group|| + 1e-6)).
 * grads scaled by `grad_scale` first (1/world_size after an RCCL sum).
 * Groups are contiguous ranges [goff[i], goff[i+1]) of the flat buffers.
 * ws: fp32 workspace of >= 64 * n_groups floats.  Up to 8 groups; two
 * launches (per-group partial sums, then coefficient + update). */
int gs_clip_sgd(int32_t n_groups, const int64_t* goff_host, float* params,
                float* grads, float grad_scale, float max_norm, float lr,
                float* ws, void* stream);

/* f32 → bf16 (RNE) cast, n elements. */
int gs_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream);

/* ------------------------------------------------------- training runtime
 * One supervised step of the reference loop (utils.py:144-191 without
 * extend_nodes): GraphSage forward over a packed sample, Classification +
 * NLL mean, backward into the flat gradient buffer, then (separate call, so
 * the caller can all-reduce gradients in between) clip_grad_norm_(max_norm)
 * per model and SGD.  Flat parameter layout:
 *   [sage_layer1.weight | ... | sage_layerL.weight | layer.0.weight | layer.0.bias]
 * Device pointers stay owned by the caller. */
typedef struct {
    int32_t n_layers, hidden, n_classes;
    int32_t agg;        /* gs_agg */
    int32_t gcn;
    int32_t feat_dtype; /* gs_dtype of X */
    int64_t feat_dim, feat_ld;
    const void* X;          /* [N, feat_ld] raw features                 */
    const int64_t* row_ptr; /* device CSR (optional: packs carry absolute entries) */
    const int32_t* col;
    const int32_t* labels;  /* [N] class ids                             */
    float* params;          /* flat, gs_trainer_n_params floats          */
    float* grads;
    float lr, max_norm;     /* reference: 0.7, 5 (utils.py:136, :186)    */
} gs_trainer_config;

typedef struct gs_trainer gs_trainer;
int gs_trainer_create(const gs_trainer_config* cfg, gs_trainer** out);
void gs_trainer_destroy(gs_trainer* t);
int64_t gs_trainer_n_params(const gs_trainer* t);
/* Workspace bytes for a sample with hop_sizes[L][4] = (n_dst, n_pos, n_src,
 * n_nbr) per hop; -1 on error. */
int64_t gs_trainer_ws_bytes(gs_trainer* t, const int64_t* hop_sizes);
/* pack: the device copy of gs_sample_pack; offsets: gs_pack_layout.off
 * flattened [GS_MAX_HOPS][GS_PK_NFIELDS]; roots: [n_roots] device ids.
 * Writes loss[0] and overwrites every gradient. */
int gs_trainer_forward_backward(gs_trainer* t, const int32_t* pack,
                                const int64_t* hop_sizes, const int64_t* offsets,
                                const int32_t* roots, int64_t n_roots, void* ws,
                                int64_t ws_bytes, float* loss, void* stream);
/* Split form of forward_backward for overlapping consecutive steps: the
 * layer-1 gather-aggregate of a batch (which reads only X and the pack) into
 * trainer slot 0..2 on any stream, then the rest of the step reading that
 * slot.  The caller orders them (event) and keeps a slot until the step that
 * reads it has finished its backward.  gs_trainer_gather_reserve allocates
 * the three slots for up to max_rows layer-1 destinations; with max_fanout
 * > 0 (the last hop's fanout, which bounds every sampled neighbourhood)
 * gs_trainer_gather runs as two launches: the positions resolved into
 * padded neighbour ids, then the row gather through them (bitwise the same
 * aggregate, without the index chain in the gather); that gather also copies
 * each destination's own feature row beside its aggregate (slot rows
 * [self | agg] of 2F, so the layer-1 GEMMs read no self index;
 * GS_TOPT_SELF_ROWS = 0 at reserve time keeps F-wide slots). */
int gs_trainer_gather_reserve(gs_trainer* t, int64_t max_rows, int32_t max_fanout);
int gs_trainer_gather(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                      const int64_t* offsets, int32_t slot, void* stream);
int gs_trainer_forward_backward_gathered(gs_trainer* t, const int32_t* pack,
                                         const int64_t* hop_sizes, const int64_t* offsets,
                                         const int32_t* roots, int64_t n_roots, int32_t slot,
                                         void* ws, int64_t ws_bytes, float* loss, void* stream);
/* Forward alone — GraphSage.forward (models.py:241-269) as get_gnn_embeddings
 * (utils.py:59-78) and evaluate (utils.py:27, :39) call it: the batch's
 * [n_roots, hidden] embeddings (row i = root i) are written to out
 * (contiguous rows).  No loss head, backward or gradient writes.  The
 * _gathered form reads the layer-1 aggregate from gather slot `slot`. */
int gs_trainer_forward(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                       const int64_t* offsets, void* ws, int64_t ws_bytes, float* out,
                       void* stream);
int gs_trainer_forward_gathered(gs_trainer* t, const int32_t* pack, const int64_t* hop_sizes,
                                const int64_t* offsets, int32_t slot, void* ws,
                                int64_t ws_bytes, float* out, void* stream);
/* grads *= grad_scale, clip per model, SGD.  ws: >= 130 floats. */
int gs_trainer_update(gs_trainer* t, float grad_scale, float* ws, void* stream);
/* Single-process update (no all-reduce between the step and the update):
 * clip per model + SGD from the gradient-norm partials the last forward/
 * backward left with its gradient reductions (one launch), or as
 * gs_trainer_update(t, 1, ...) when that backward could not produce them. */
int gs_trainer_update_local(gs_trainer* t, void* stream);
/* Measurement only: record HIP events on the launch stream around the next
 * `capacity` layer-1 launches — the fused gather + linear kernel when
 * the gather-aggregate; gs_trainer_agg_times
 * synchronises and returns their durations (ms). */
int gs_trainer_time_agg(gs_trainer* t, int64_t capacity);
int64_t gs_trainer_agg_times(gs_trainer* t, float* ms, int64_t cap);
/* The same timers per site: 0 the layer-1 gather as above, 1 the layer-1
 * SageLayer forward GEMM (gs_sage_linear_fwd, unfused path), 2 the layer-1
 * weight-gradient GEMM of the fused backward (linear_dw slabs, before their
 * sum), 3 the fused top layer + loss head launch (2-layer models), 4 the
 * slab-sum pair launch (the layer-1 and layer-2 weight-gradient sums of the
 * fused top path).
 * gs_trainer_time_kernels arms the sites in site_mask (bit s = site
 * s) for their next `capacity` launches and disarms the others;
 * gs_trainer_time_agg(t, n) == gs_trainer_time_kernels(t, 1, n).  Every
 * armed launch is an event-bound hipExtLaunchKernel, which costs the stream
 * a little (a few microseconds of idle queue on either side of it): time the
 * GEMM sites in their own steps, not the measured ones.
 * gs_trainer_time_kernels_every times one launch in `every` of each armed
 * site (the every-th, 2·every-th, ... launch since arming), so a measured
 * window pays the event cost on a fraction of its steps. */
int gs_trainer_time_kernels(gs_trainer* t, int32_t site_mask, int64_t capacity);
int gs_trainer_time_kernels_every(gs_trainer* t, int32_t site_mask, int64_t capacity, int64_t every);
int64_t gs_trainer_kernel_times(gs_trainer* t, int32_t site, float* ms, int64_t cap);
/* For a stamped site (1-4): per timed launch,
 * four floats in us — span (first workgroup start .. last end), mean and max
 * workgroup duration, and the spread of workgroup starts; -1 for a launch
 * timed by events.  Returns the launches written, -1 on error. */
int64_t gs_trainer_kernel_block_stats(gs_trainer* t, int32_t site, float* us4, int64_t cap);
/* The raw per-workgroup stamps (100 MHz s_memrealtime ticks; 0 = none) of
 * stamped launch `launch` of `site`: kStampBlocks (1024) entries each into
 * start and end.  Returns the entries written, 0 for an unstamped launch. */
int64_t gs_trainer_kernel_stamps(gs_trainer* t, int32_t site, int64_t launch, uint64_t* start, uint64_t* end);
/* Demangled name of the kernel timer site `site` timed since it was last
 * armed ("" before its first timed launch) — the variant actually launched. */
const char* gs_trainer_kernel_name(const gs_trainer* t, int32_t site);
/* The flat gradient buffer (cfg.grads), gs_trainer_n_params floats. */
float* gs_trainer_grads(const gs_trainer* t);
/* Parity capture (tests): after each of the next max_steps training steps
 * (gs_trainer_forward_backward[_gathered], inside gs_runner_run too), copy on
 * the step's stream the step's [n_roots, hidden] root embeddings (the top
 * SageLayer's output, models.py:241-269) to emb + i * emb_stride and the flat
 * gradient as the step's backward left it — before its clip_grad_norm_ and
 * SGD (utils.py:184-187) — to grads + i * gs_trainer_n_params.  Either buffer
 * may be NULL; max_steps 0 disarms.  gs_trainer_captured: steps copied. */
int gs_trainer_capture(gs_trainer* t, float* emb, int64_t emb_stride, float* grads, int64_t max_steps);
int64_t gs_trainer_captured(const gs_trainer* t);
/* Deferred clip + SGD for a caller's own data-parallel loop (utils.py:184-187
 * per rank after the gradient sum), as gs_runner_run runs it with a
 * communicator: with on = 1, each gs_trainer_update(t, 1/W, ...) after the
 * all-reduce leaves the update pending — one launch computes the summed
 * gradient's clip-norm partials and W1's speculative update S = W1 - lr*g/W —
 * and the next forward applies the clip + SGD in its prologue (the fold of
 * those partials with scale 1/W).  on = 0 applies a pending update and leaves
 * deferred mode, so the flat parameters are current again.  *active (may be
 * NULL): 1 when deferring took effect (the step's shape allows it: 2 layers,
 * fused top launch and backward, 16-byte feature rows), else 0 and every
 * update runs at once.  Not inside a runner loop. */
int gs_trainer_defer(gs_trainer* t, int32_t on, int32_t* active, void* stream);
/* Trainer options (gs_trainer_set_option, value 0 / 1; not inside a runner
 * loop; all default 1 except GS_TOPT_TOP_PAIR, default 0).  Each alternative
 * exists for the tests that compare it with the default.  fused_bwd, self_rows and defer_update compute bitwise the
 * default's results; top_launch matches them within fp32 rounding of the
 * k order (its split-K partial sums are added in a fixed, different order):
 *   GS_TOPT_FUSED_BWD     1: layers >= 2 backward in fused launches
 *   GS_TOPT_TOP_LAUNCH    1: a 2-layer step's layer 2 + loss head + dIn2 in one launch
 *   GS_TOPT_SELF_ROWS     1: gather slots hold [self | agg] rows (next gs_trainer_gather_reserve)
 *   GS_TOPT_DEFER_UPDATE  1: runner loops defer each step's clip + SGD into the next step
 *   GS_TOPT_TOP_PAIR      1: the top launch on two blocks per 4 roots (<= 16 classes), each with
 *                         half of W2, the partial logits exchanged in the launch; within fp32
 *                         rounding of the one-block form, deterministic; default 0 (the
 *                         layer-2 backward then adds two dIn partials: neutral per step) */
enum { GS_TOPT_FUSED_BWD = 0, GS_TOPT_TOP_LAUNCH = 1, GS_TOPT_SELF_ROWS = 2, GS_TOPT_DEFER_UPDATE = 3,
       GS_TOPT_TOP_PAIR = 4 };
int gs_trainer_set_option(gs_trainer* t, int32_t opt, int32_t value);

/* ------------------------------------------------------- RCCL communicator
 * One communicator per data-parallel rank for the gradient all-reduce of the
 * native runner (utils.py:184-187 per rank, then an average over ranks).
 * Rank 0 creates the id; the caller broadcasts its 128 bytes. */
int gs_comm_unique_id(uint8_t id[128]);
int gs_comm_create(const uint8_t id[128], int32_t n_ranks, int32_t rank, void** comm);
void gs_comm_destroy(void* comm);
/* In-place sum over ranks of n fp32 values on `stream`. */
int gs_comm_allreduce_sum(void* comm, float* buf, int64_t n, void* stream);

/* ------------------------------------------------------- pipeline runner
 * The reference's epoch loop over batches (utils.py:144-191 called from
 * main.py per epoch) as a native pipeline: S sampler threads (stream w owns
 * batches w, w+S, ... and its own rng — S = 1 is the reference's single
 * random stream) fill rings of pinned pack buffers with gs_sample_pack_run;
 * gs_runner_run consumes the batches in order, issuing on `stream` the pack's
 * H2D copy (two device buffers, reused in stream order), forward_backward,
 * the optional all-reduce and the update.  Sampler threads make no HIP calls;
 * the calling thread recycles a pinned slot once its copy event completes.
 * The rngs, graph and trainer are borrowed and must outlive the runner;
 * `batches` (n_batches x batch int64 ids) is copied. */
typedef struct {
    const gs_graph* graph;
    gs_trainer* trainer;
    const int64_t* batches;
    int64_t n_batches, batch;
    const int32_t* fanouts;
    int32_t n_hops;
    int32_t flags;          /* GS_SAMPLE_* */
    int32_t n_streams;
    gs_rng* const* rngs;    /* [n_streams] */
    int32_t depth;          /* pinned slots per stream (>= 1) */
    void* comm;             /* gs_comm_create handle or NULL */
    int32_t world;          /* gradient scale 1/world after the all-reduce */
    /* Inference (get_gnn_embeddings, utils.py:59-78): when non-NULL every step
     * is gs_trainer_forward_gathered into embed_out + b * batch * embed_ld
     * ([n_batches * batch, embed_ld] fp32, embed_ld = hidden): no loss,
     * backward, all-reduce or update. */
    float* embed_out;
    int64_t embed_ld;
    /* Inference only: reference batches per device launch (<= 1: one).  Step
     * u then samples batches u*merge .. u*merge+merge-1 on stream u % S into
     * one pack (gs_sample_pack_run_multi) and runs one forward over all of
     * them; gs_runner_run counts these merged steps. */
    int32_t merge;
    /* hold != 0: the sampler threads start no batch at or past the release
     * mark (initially 0) until gs_runner_release raises it, so a measurement
     * can prove that none of its batches was sampled before its clock
     * started.  hold == 0: the mark is unbounded (sampling starts at create). */
    int32_t hold;
    /* Gradient all-reduce buckets with a communicator (training only): 1 (or
     * 0) = one in-place all-reduce of the flat gradient after the backward;
     * 2 = the upper layers' and classifier's gradients [W2 .. | Wc | bc]
     * (final once the layers >= 2 backward has run) all-reduced on a comm
     * stream under the layer-1 weight-gradient GEMM, then W1 after them on
     * the same comm stream (one stream order on every rank).  Same sums
     * either way (the buckets are disjoint ranges). */
    int32_t ar_buckets;
    /* Helper threads per sampler stream (gs_team): lower per-batch latency
     * for the same draws — for few streams (the reference-sequence S = 1
     * mode) or a cold pipeline.  0: none. */
    int32_t helpers;
    /* warm != 0: before gs_runner_create returns, every sampler thread (and
     * its helpers) samples one throwaway batch — the stream's last batch,
     * drawn from a copy of its rng, so no stream advances and no batch is
     * sampled ahead — so that no measured batch pays the first-use costs of
     * the thread's sampling context (allocation, page faults). */
    int32_t warm;
    /* device_sampler != 0 (training and merge <= 1 inference): the S streams
     * sample on the GPU — one gs_dsampler per stream, each on
     * its own HIP stream, seeded from rngs[w] — and write every pack straight
     * into the device pack ring: no sampler threads, pinned slots or pulls.
     * Stream w samples batches w, w+S, ... exactly as the host sampler would
     * (same packs, same stream consumption); batch b+S is sampled while the
     * device runs the steps before it.  The rngs are written back at
     * gs_runner_sync_rngs and gs_runner_destroy. */
    int32_t device_sampler;
} gs_runner_config;

typedef struct {
    int64_t steps;          /* steps issued since the last reset */
    double wait_s;          /* host time blocked, = the three parts below */
    double issue_s;         /* host time issuing launches */
    double sample_s;        /* summed sampler-thread time of those batches */
    double hop_sizes[4 * GS_MAX_HOPS]; /* summed (n_dst, n_pos, n_src, n_nbr) */
    double wait_sample_s;   /* ... on a not-yet-sampled batch */
    double wait_ring_s;     /* ... on the step three batches back (ring entry reuse) */
    double wait_gather_s;   /* ... on this batch's side-stream pull + gather */
    double fwd_bwd_s, update_s; /* parts of issue_s */
    double max_step_s;      /* longest single step (wait + issue) */
    int64_t lookahead_misses; /* steps whose batch was not issued one step ahead */
} gs_runner_stats;

typedef struct gs_runner gs_runner;
int gs_runner_create(const gs_runner_config* cfg, gs_runner** out);
/* Issue the next n_steps steps (GPU work asynchronous on `stream`); fails
 * with the sampler's error (e.g. GS_EEMPTY) or GS_ERANGE past n_batches. */
int gs_runner_run(gs_runner* r, int64_t n_steps, float* loss, void* stream);
int gs_runner_stats_get(const gs_runner* r, gs_runner_stats* out);
void gs_runner_stats_reset(gs_runner* r);
/* Raise the release mark (cfg.hold): batches < mark may now be sampled.
 * Returns GS_EINVAL when mark is lower than the current one. */
int gs_runner_release(gs_runner* r, int64_t mark);
/* Progress counters: *sampled = batches (steps) whose sampling has
 * completed, *consumed = steps issued by gs_runner_run; sampled - consumed
 * is the number of batches sampled ahead of the device at this instant. */
int gs_runner_progress(const gs_runner* r, int64_t* sampled, int64_t* consumed);
/* device_sampler runners: copy every device stream's state back into its
 * rngs[w] (waits for the stream's sampling in flight; the state then
 * includes every batch sampled so far, consumed or not — as the host
 * sampler threads' rngs do).  Host-sampler runners: no-op. */
int gs_runner_sync_rngs(gs_runner* r);
void gs_runner_destroy(gs_runner* r);

#ifdef __cplusplus
}
#endif
#endif /* GRAPHSAGE_AMD_H */

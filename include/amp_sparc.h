/*
 * amp_sparc.h — C ABI of the MI355X (gfx950) AMP/VAMP spatial-modulation detector.
 *
 * Drop-in boundary for the hot path of AhmedKishki/AMP-SPARC-SpatialModulation.
 * The reference exposes no FFI: its boundary is the Python class surface
 * (VAMP / BAMP / SCAMP / Loss).  The host package
 * `amp-sparc-spatialmodulation_amd/` keeps that surface and binds these entry
 * points through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every array argument is a DEVICE pointer
 *    owned by the caller; nothing is retained after a call returns.
 *  - complex64 arrays are interleaved {re, im} float pairs (torch.complex64 layout).
 *    Batched vectors are row-major [B][len] (the reference's [B, len, 1]).
 *  - Every call is asynchronous on `stream` (a hipStream_t passed as void*), makes
 *    no allocation and no host synchronisation, so it may be captured in a hipGraph.
 *    Results that the host needs (iteration count, error counters) are written to
 *    small device structs the caller copies back once.
 *  - Return value: 0 on success, a negative AMP_E* code otherwise;
 *    amp_last_error() returns a message for the last failure on this thread.
 *    The reference raises Python exceptions instead (AssertionError in
 *    config.py:40-44, ValueError on bad reshapes); the host layer maps a
 *    non-zero code to a Python exception.  NaN outputs are a legal state
 *     and never an error.
 */
#ifndef AMP_SPARC_H
#define AMP_SPARC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMP_OK 0
#define AMP_E_ARG (-1)       /* bad argument / unsupported shape */
#define AMP_E_WORKSPACE (-2) /* workspace too small */
#define AMP_E_LAUNCH (-3)    /* HIP launch failure */

#define AMP_MAX_K 64         /* 64-QAM (BASELINE cfg5; the reference's own Config stops at 16, config.py:44)
                              * sizes: K in {1, 2, 4, 8, 16, 64} */

/* Constellation of Config (config.py:78-118): unit-power points in float32 (for the
 * denoiser) and float64 (for the MAP decision, loss.py:295), plus gray labels. */
typedef struct amp_constellation {
    int32_t K;
    int32_t symbol_bits;          /* int(log2 K), config.py:119 */
    float re[AMP_MAX_K];
    float im[AMP_MAX_K];
    double re64[AMP_MAX_K];
    double im64[AMP_MAX_K];
    int32_t gray[AMP_MAX_K];
} amp_constellation;

/* System dimensions (Config, config.py:49-71, 132-144; sparc mode).
 * N = Nt*Lin (unknowns per trial), n = Nr*Lout (observations per trial),
 * L = Na*Lin sections of M = Nt/Na positions each. */
typedef struct amp_dims {
    int32_t B, Nt, Na, Nr, Lin, Lout;
    int32_t N, n, L, M;
} amp_dims;

/* Per-forward result written by the detector drivers (device memory). */
typedef struct amp_status {
    int32_t T;          /* executed iterations (t+1 at the early-exit break, vamp.py:185) */
    int32_t nan_state;  /* 1 when the last iteration produced NaN sections (float64 underflow rule) */
    int32_t stopped;    /* 1 when the allclose early exit fired */
    int32_t gemm;       /* the GEMM arithmetic that ran: AMP_ARITH_* (0: not reported) */
    float last_scalar[4]; /* VAMP: sigma2_tilde, alpha, sigma2, dxdr of the last iteration */
} amp_status;

/* amp_status.gemm: the arithmetic of the engine's GEMMs in the forward that wrote the record */
#define AMP_ARITH_F32 1      /* float32 operands and accumulation (f32 MFMA / tiles) */
#define AMP_ARITH_BF16X3 2   /* three bf16 pieces per f32 operand (24 bits), six products, f32 accumulation */
#define AMP_ARITH_FP16X2 3   /* two fp16 pieces per scaled operand (22 bits), three products (opt-in) */
#define AMP_ARITH_INT8X4 4   /* four int8 digits per block-fixed-point operand (31 bits), exact int32 sums (opt-in) */

/* Error counters of Loss.error_rate (loss.py:67-179), written by amp_map_decide_count. */
typedef struct amp_counts {
    int64_t ier, ser;           /* index / gray-label mismatches over Ns sections (loss.py:165-166) */
    int64_t iber, sber;         /* bit mismatches (loss.py:168, 172) */
    int64_t ver, verf, verm, verL;  /* channel uses with any wrong entry (loss.py:133-136) */
    int64_t fer;                /* trials with any wrong entry (loss.py:150) */
    double mse, msef, msem, mseL;   /* sum |xmmse - x|^2, all / lin 0 / Lin//2 / last (loss.py:116-119) */
} amp_counts;

/* ---- VAMP (SVD form) — replaces VAMP.forward (vamp.py:159-187) with its
 *      Tracker (vamp.py:12-28) and T x VAMPLayer.forward (vamp.py:56-94). ---- */
typedef struct amp_vamp_args {
    const void* U;      /* c64 [n][k]  (torch.linalg.svd output, vamp_model.py:58) */
    const void* s;      /* f32 [k] */
    const void* Vh;     /* c64 [k][N] */
    const void* y;      /* c64 [B][n] */
    int32_t k;          /* min(n, N) */
    int32_t max_iter;   /* config.N_Layers */
    int32_t engine;     /* amp_vamp_run only: AMP_ENGINE_AUTO / _LAUNCHES / _PERSISTENT */
    int32_t gemm;       /* persistent-engine GEMM arithmetic: AMP_GEMM_AUTO / _F32 / _X3 / _H2 */
    double noise_var;   /* Na/Nr/SNR (vamp.py:179) */
    double sparsity;    /* Na/Nt (vamp.py:155) */
    void* r;            /* out c64 [B][N]: decision input T.r (vamp.py:187) */
    void* xmmse;        /* out c64 [B][N] */
    void* var;          /* out f32 [B][N] */
    void* status;       /* out amp_status (device) */
    void* ws;           /* workspace, amp_vamp_workspace_bytes() bytes */
    size_t ws_bytes;
} amp_vamp_args;

/* Engines of amp_vamp_run (same results up to f32 summation order):
 *  LAUNCHES   three launches per iteration (the layer-level path below);
 *  PERSISTENT one launch for the whole loop (co-residency checked): each workgroup keeps 16 trials'
 *             state in LDS across iterations, one grid barrier per iteration carries the
 *             batch-global scalars (needs k == N, N % 32 == 0, N <= 256, M <= 64 and
 *             ceil(B/16) workgroups co-resident: B <= 16 x #CUs);
 *  AUTO       PERSISTENT when eligible, else LAUNCHES. */
/* Persistent-engine GEMM arithmetic (amp_vamp_args.gemm):
 *  F32   v_mfma_f32_16x16x4_f32 on the real expansion of each operator;
 *  X3    split precision: every f32 operand as three bf16 pieces (all 24 bits: the reference's
 *        c64 operand precision), six bf16 MFMA products per product (terms below 2^-24 relative
 *        dropped), f32 accumulation — the f32 GEMM's accuracy at 2.7x the MFMA rate (needs
 *        k == N, N % 64 == 0 and 160 KB of LDS);
 *  H2    OPT-IN, narrower than the reference: every A row scaled by its own power of two, every
 *        value as two fp16 pieces (22 significant bits), three fp16 MFMA products per product
 *        (the 2^-22 lo.lo term dropped), f32 accumulation, the scales taken off exactly; the
 *        operators must have entries of magnitude < 4 (SVD factors: <= 1; larger entries give
 *        non-finite results, never silently wrong ones); same shape constraints as X3;
 *  I8    int8x4 block fixed point on the integer matrix cores: every A row and every operator
 *        column scaled by its own power of two, every value as a 31-bit integer in four
 *        balanced 8-bit digits, the ten digit products of levels 0-3 exact in int32
 *        (v_mfma_i32_16x16x64_i8), the levels combined in f32: 31 bits per element relative to
 *        its row's / column's maximum (>= 24 bits down to 2^-7 of it), dropped terms < 2^-30 of
 *        (row max . column max); on the cfg4 GEMM 23x closer to a float64 sum than an f32 sum
 *        (amp_persist.h gemm_i8); a non-finite A row gives a NaN result row; same shape
 *        constraints as X3, one workgroup per CU.  Its different rounding moves the allclose
 *        early exit (vamp.py:185) where that exit is decided by rounding: at three cfg4-QPSK
 *        1 dB golden points it stops at 18 / 16 / 14 iterations where the reference runs to 20
 *        (VER / SER within 1e-3; tests/test_gpu_vamp.py T_DIVERGENCE);
 *  AUTO  X3 where the planes fit, else F32 (environment AMP_VAMP_GEMM=f32 keeps F32,
 *        AMP_VAMP_GEMM=h2 picks H2). */
#define AMP_GEMM_AUTO 0
#define AMP_GEMM_F32 1
#define AMP_GEMM_X3 2
#define AMP_GEMM_H2 3
#define AMP_GEMM_I8 4

#define AMP_ENGINE_AUTO 0
#define AMP_ENGINE_LAUNCHES 1
#define AMP_ENGINE_PERSISTENT 2

/* The engine amp_vamp_run will use for this shape on the current device (LAUNCHES or
 * PERSISTENT), or AMP_E_ARG when `engine` is PERSISTENT and the shape is not eligible. */
int amp_vamp_select_engine(const amp_dims* d, int32_t k, int32_t engine);
/* The arithmetic the persistent engine will use for this shape: AMP_GEMM_X3, AMP_GEMM_H2,
 * AMP_GEMM_I8 or AMP_GEMM_F32 (AMP_E_ARG when `gemm` is X3 / H2 / I8 and the shape does not fit). */
int amp_vamp_select_gemm(const amp_dims* d, int32_t k, int32_t gemm);
/* Diagnostic: a persistent-engine forward that stamps s_memtime per workgroup, iteration and
 * phase into trace (device, nwg * max_iter * 10 + 4 * nwg uint64; layout in amp_vamp.hip). */
int amp_vamp_persist_trace(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* trace,
                           void* stream);
/* Diagnostic (bench.py): while on != 0, every persistent VAMP launch records a HIP event pair
 * around its vamp_persist kernel on its stream; amp_debug_persist_time synchronises them, returns
 * how many launches were timed and their mean duration in ms, and clears the record. */
int amp_debug_persist_timing(int32_t on);
int amp_debug_persist_time(int32_t* n, float* mean_ms);
size_t amp_vamp_workspace_bytes(const amp_dims* d, int32_t k, int32_t max_iter);
int amp_vamp_run(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream);
/* Layer-level pieces of amp_vamp_run: prepare = Tracker (vamp.py:13-28);
 * iterate(t) = one VAMPLayer.forward + the allclose test of vamp.py:185 (no-op once stopped);
 * finalize = iteration count and NaN bookkeeping for the returned Loss. */
int amp_vamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream);
int amp_vamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, int32_t t, void* stream);
int amp_vamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, void* stream);
/* VAMP.forward + Loss.error_rate in one call (vamp.py:159-187 then loss.py:67-179): the
 * forward of amp_vamp_run and the MAP decision on its r (vamp.py:187) with every counter of
 * amp_map_decide_count.  On the PERSISTENT engine the decision runs in the same launch, on
 * the rows each workgroup still holds in LDS (the counters are identical to
 * amp_map_decide_count's).  Returns AMP_E_ARG when the shape is not persistent-eligible (use
 * amp_vamp_run + amp_map_decide_count). */
typedef struct amp_vamp_decide_args {
    const void* x;        /* c64 [B][N] transmitted vector */
    const void* sym;      /* int64 [B*L] true gray labels (data.py:89) */
    const void* idx;      /* int64 [B*L] true flat nonzero indices (data.py:90) */
    int32_t ibits_trunc;  /* ceil(log2(Lin*B*Na)) (loss.py:20) */
    int32_t pad;
    void* counts;         /* out amp_counts (device) */
    void* host_record;    /* optional (NULL: none): a 256-byte page-locked host buffer mapped for the
                           * device (hipHostMalloc / torch pin_memory).  amp_vamp_detect_count on the
                           * persistent engine then also writes the forward's amp_status at byte 0
                           * and its amp_counts at byte 64 there (system-scope stores from the last
                           * kernel of the forward), so the caller needs no device-to-host copy: the
                           * record is valid once the stream has passed the forward.  Ignored by
                           * the other entry points. */
} amp_vamp_decide_args;
int amp_vamp_detect_count(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                          const amp_vamp_decide_args* dec, void* stream);
/* `epochs` independent forwards of d->B trials each that share ONE channel (U, s, Vh) — the
 * epochs of one `res` block of Model.simulate (vamp_model.py:55-61: the channel is redrawn only
 * when i % res == 0) — side by side in one persistent launch.  Each epoch keeps its own
 * batch-global scalars (mean var, max|xi|, allclose; vamp.py:85, 112, 185) and early exit, so
 * the results equal `epochs` sequential amp_vamp_detect_count calls.  y, r, xmmse, var, x, sym,
 * idx hold the epochs' rows back to back ([epochs * B] rows); status -> amp_status[epochs],
 * dec->counts -> amp_counts[epochs]; workspace: amp_vamp_epochs_workspace_bytes.  Needs the
 * persistent engine with B % 16 == 0 and epochs <= amp_vamp_max_epochs (one workgroup of 16
 * trials per CU; two per CU at N = 64 only in the diagnostic build with AMP_EPOCHS_TWO_PER_CU=1). */
/* ---- Trial sharding across ranks (SURVEY §8(e) exact-compat mode) ----
 * One batch of B_global trials split over ranks (rank r holds a contiguous slice of d->B rows);
 * every per-iteration batch-global value of VAMP.forward (var.mean() vamp.py:85, the float64
 * max|xi| shift vamp.py:112, torch.allclose vamp.py:185, and the rare path's exact values) is
 * all-reduced through a caller-registered hook between launches, so each rank follows the
 * trajectory of the whole-batch forward.  The hook all-reduces `count` float64 words at the
 * device pointer `buf` in place, ordered on `stream` (e.g. an RCCL ncclAllReduce on that stream,
 * or torch.distributed.all_reduce); it returns 0 on success.  It is called 4 times per
 * iteration on every rank (no data-dependent calls, no host synchronisation inside).
 * Failure semantics: a hook that fails must still take part in its collective (e.g. with NaN
 * words) and return nonzero; the driver keeps making every later call of the forward, so the
 * ranks' collectives stay matched, and then returns AMP_E_LAUNCH on that rank.  The poisoned
 * words reach every rank; the caller decides collectively whether to discard the forward
 * (vamp.ShardHook._run_hooked all-reduces an error flag and raises on every rank). */
enum { AMP_ALLREDUCE_SUM = 0, AMP_ALLREDUCE_MAX = 1 };
typedef int (*amp_allreduce_fn)(void* buf, int64_t count, int32_t op, void* stream, void* ctx);
int amp_set_allreduce_hook(amp_allreduce_fn fn, void* ctx);
/* The same split on the PERSISTENT engine (one launch per forward, no per-iteration host calls):
 * every rank's grid publishes its per-iteration batch partials into ONE shared exchange buffer at
 * its workgroups' global indices and every workgroup of every rank reduces all of them in the
 * whole batch's order, so every rank derives the whole-batch forward's scalars bit for bit
 * (vamp.py:85, 112, 185) and its rows of r / xmmse / var equal the whole-batch forward's.
 * xbuf: device memory every rank's kernel reads and writes (on one GPU: one allocation shared by
 * grids on different streams, which must be co-resident together; across GPUs it would be
 * peer-mapped memory, whose coherence this build does not provide: one device only), at least
 * amp_vamp_shard_xbuf_bytes(B_global, max_iter) bytes; amp_vamp_shard_reset zeroes its barrier
 * words, once before every forward after every rank's previous forward has finished.  gen: the
 * same value on every rank, a new one for every forward on this buffer (it tags the exchange
 * records).  This rank detects trials [row_offset, row_offset + d->B) (row_offset a multiple of 16,
 * d->B too except for the last rank); y / r / xmmse / var / x / sym / idx hold its rows only;
 * dec->counts gets its rows' counters (sum them over the ranks).  Replaces amp_vamp_run_sharded
 * for the shapes the persistent engine takes (vamp.py:159-187). */
typedef struct {
    void* xbuf;
    size_t xbuf_bytes;
    int32_t B_global;
    int32_t row_offset;
    uint32_t gen;
    int32_t pad;
} amp_vamp_shard;
size_t amp_vamp_shard_xbuf_bytes(int32_t B_global, int32_t max_iter);
int amp_vamp_shard_reset(void* xbuf, void* stream);
int amp_vamp_detect_count_shard(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                const amp_vamp_decide_args* dec, const amp_vamp_shard* sh, void* stream);
/* amp_vamp_run on this rank's slice (launch engine) with the batch scalars all-reduced; workspace
 * as amp_vamp_workspace_bytes(d, ...) for the slice.  Decide with amp_map_decide_count_rows. */
int amp_vamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, int32_t B_global,
                         void* stream);

size_t amp_vamp_epochs_workspace_bytes(const amp_dims* d, int32_t k, int32_t max_iter, int32_t epochs);
/* Diagnostic: byte offsets inside the epochs workspace of the persistent engine's exchange
 * records: out[0] the per-iteration granule pairs ([max_iter][epochs * ceil(B/16)] x 32 B:
 * {sum var f64, not-close u32, tag u32}, {max|xi| f32, min section max f32, 0, tag}), out[1] the
 * rare-path float64 words, out[2] the barrier words, out[3] the per-workgroup counter records,
 * out[4] y~ ([epochs * B][2k] floats; also the single-forward workspace's, epochs = 1). */
int amp_vamp_debug_offsets(const amp_dims* d, int32_t k, int32_t max_iter, int32_t epochs, uint64_t* out);
/* Diagnostic: every later persistent VAMP launch of this process writes its per-iteration state
 * to buf (device, float32: [max_iter][nwg][5][16][2N]: w after GEMM1's epilogue, r after GEMM2's,
 * xmmse after the denoiser, then var (columns < N) and the waves' float64 var sums (row 0,
 * columns N ..), then the denoiser's exclusive section sum and variance sum (columns < N / >= N), per
 * workgroup's 16 rows); null turns it off. */
int amp_vamp_debug_dump(void* buf);
/* The most epochs of d->B trials one launch holds on this device (0: not persistent-eligible). */
int amp_vamp_max_epochs(const amp_dims* d, int32_t k);
/* The same for a given persistent GEMM arithmetic (amp_vamp_args.gemm).  One workgroup per CU;
 * the diagnostic build with AMP_EPOCHS_TWO_PER_CU=1 allows two where that arithmetic has the
 * two-per-CU build (the split-precision forms at N = 64). */
int amp_vamp_max_epochs_gemm(const amp_dims* d, int32_t k, int32_t gemm);
/* 1 when amp_vamp_detect_count_epochs_ch takes ONE CHANNEL PER EPOCH for this config and GEMM
 * arithmetic (the bf16x3 / int8x4 engine and n == 2 k), else 0 (then a chunk of epochs must share
 * one channel, as amp_vamp_detect_count_epochs). */
int amp_vamp_epochs_ch_eligible(const amp_dims* d, int32_t k, int32_t gemm);
int amp_vamp_detect_count_epochs(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                 const amp_vamp_decide_args* dec, int32_t epochs, void* stream);
/* The same with ONE CHANNEL PER EPOCH — Model.simulate at the reference's default res = 1
 * (vamp_model.py:45, 56-58: a new channel and its SVD every epoch): epoch e reads U at
 * a->U + e * U_stride, s at a->s + e * s_stride and Vh at a->Vh + e * Vh_stride (elements: complex64
 * for U / Vh, float for s; all zero = one shared channel, as amp_vamp_detect_count_epochs).  Needs the
 * bf16x3 (AUTO) or int8x4 engine; workspace: amp_vamp_epochs_workspace_bytes (it always holds one
 * operator set per epoch).  Replaces `epochs` calls of VAMP.forward with their own channels. */
int amp_vamp_detect_count_epochs_ch(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a,
                                    const amp_vamp_decide_args* dec, int32_t epochs, int64_t U_stride,
                                    int64_t s_stride, int64_t Vh_stride, void* stream);
/* Measurement helper (not graph-safe: synchronises): one forward with hipEvents between the
 * launches, in milliseconds.  LAUNCHES engine: ms_out[4] = mean GEMM1 / GEMM2+denoiser /
 * reduction kernel time per executed iteration and the whole forward.  PERSISTENT engine
 * (as a->engine selects it): prepare (weights + y~ GEMM), the vamp_persist launch, 0, total. */
int amp_vamp_profile(const amp_dims* d, const amp_constellation* c, const amp_vamp_args* a, float* ms_out,
                     void* stream);

/* ---- BAMP — replaces BAMP.forward (bamp.py:116-143) with BAMPLayer.forward
 *      (bamp.py:48-64) and its per-element-tau denoiser (bamp.py:66-77). ---- */
typedef struct amp_bamp_args {
    const void* H;      /* c64 [n][N] */
    const void* y;      /* c64 [B][n] */
    int32_t max_iter;
    int32_t denoiser;   /* 0: segmented block denoiser (bamp.py:66-77, modes 'sparc'/'segmented');
                           1: element-wise Bayes random_denoiser (bamp.py:79-88, mode 'random'),
                              float64 with the P0 / Ps prior below */
    double noise_var;   /* Na/Nr/SNR (bamp.py:124) */
    void* xmap;         /* out c64 [B][N]: decision input T.xmap (bamp.py:142) */
    void* xmmse;        /* out c64 [B][N] */
    void* var;          /* out f32 [B][N] */
    void* status;
    void* ws;
    size_t ws_bytes;
    float P0, Ps;       /* Config.P0 / Config.Ps as float32 (bamp.py:36), denoiser 1 only */
    int32_t gemm;       /* GEMM arithmetic: AMP_GEMM_AUTO (f32 MFMA, the reference's operand
                           precision; environment AMP_BAMP_GEMM=x3 / h2 picks bf16x3 / fp16x2 where
                           N % 64 == 0 and n % 64 == 0, block-banded channels included), AMP_GEMM_F32,
                           AMP_GEMM_X3 (bf16x3 launch tiles, amp_gemm_x3.h: 24-bit operands, every
                           GEMM's A rows split once into three bf16 pieces, no range limit), or
                           AMP_GEMM_H2 (OPT-IN, 22-bit operands, amp_gemm_h2.h: every GEMM's A rows split once into
                           per-row scaled fp16 pieces; the operator pieces are scaled by 2^10, so |H|^2
                           must stay below 64, i.e. |H| < 8: beyond it a piece is inf and the detection
                           turns NaN, counted as errors, never silently wrong) */
    int32_t pad;
} amp_bamp_args;

size_t amp_bamp_workspace_bytes(const amp_dims* d, int32_t max_iter);
int amp_bamp_run(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream);
/* amp_bamp_run on one rank's slice of a trial-sharded batch (amp_vamp_run_sharded's protocol,
 * the hook of amp_set_allreduce_hook): max|xi| / min section max (bamp.py:70) and the allclose
 * count (bamp.py:140) all-reduced per iteration; decision on xmap with amp_map_decide_count_rows.
 * denoiser 0 only (the element-wise mode runs at B = 1). */
int amp_bamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, int32_t B_global,
                         void* stream);
/* Layer-level pieces of amp_bamp_run (same arguments; amp_bamp_run = prepare, iterate(t) for
 * t < max_iter, finalize): prepare = Tracker (bamp.py:13-25: the H / H^H / |H|^2 operators,
 * xmmse = 0, var = 1, z = y, u = sigma2); iterate(t) = one BAMPLayer.forward (bamp.py:48-64) +
 * the allclose(var) early exit of bamp.py:140 (a device-side no-op once it has fired);
 * finalize = the executed iterations' var into a->var and the status record. */
int amp_bamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream);
int amp_bamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, int32_t t, void* stream);
int amp_bamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_bamp_args* a, void* stream);
/* BAMPLayer.random_denoiser (bamp.py:79-88) alone (layer-level API): r c64 [count], cov f32
 * [count] -> xmmse c64, var f32; the element-wise float64 Bayes posterior of denoiser 1. */
int amp_bamp_random_denoise(const amp_constellation* c, int64_t count, const void* r, const void* cov, float P0,
                            float Ps, void* xmmse, void* var, void* stream);

/* ---- SCAMP — replaces SCAMP.forward (scamp.py:77-107) with SCAMPLayer.forward
 *      (scamp.py:43-59) and its mean-only denoiser (scamp.py:61-68). ---- */
typedef struct amp_scamp_args {
    const void* W;      /* f32 [Lout][Lin] base matrix (channel.py:80-83) */
    const void* A;      /* c64 [n][N] */
    const void* y;      /* c64 [B][n] */
    int32_t max_iter;
    int32_t engine;     /* amp_scamp_run only: AMP_ENGINE_AUTO / _LAUNCHES / _PERSISTENT (as for VAMP) */
    int32_t gemm;       /* persistent-engine GEMM arithmetic: AMP_GEMM_AUTO / _F32 / _X3 / _H2 (as for VAMP);
                           on the launch engine AMP_GEMM_X3 runs bf16x3 launch tiles (N % 64 == 0,
                           n % 64 == 0; under AUTO with AMP_SCAMP_LAUNCH_GEMM=x3), else f32 MFMA tiles */
    int32_t pad;
    double noise_var;   /* Na/Nr/SNR (scamp.py:98) */
    void* xmap;         /* out c64 [B][N] (scamp.py:107) */
    void* xmmse;        /* out c64 [B][N] */
    void* psi;          /* out f32 [B][Lin] */
    void* status;
    void* ws;
    size_t ws_bytes;
} amp_scamp_args;

size_t amp_scamp_workspace_bytes(const amp_dims* d, int32_t max_iter);
/* Engines of amp_scamp_run (same results up to f32 summation order):
 *  LAUNCHES   seven launches per iteration (the layer-level path below);
 *  PERSISTENT one launch for the whole loop: each workgroup keeps 16 trials' x, xmap, z in LDS
 *             across iterations; one granule exchange per iteration carries the batch-global
 *             max|xi| and allclose count (needs (2N, 2n) in {(128, 256), (256, 512), (256, 256)},
 *             M <= 64 and ceil(B/16) workgroups co-resident);
 *  AUTO       PERSISTENT when eligible, else LAUNCHES. */
int amp_scamp_select_engine(const amp_dims* d, int32_t engine);
int amp_scamp_run(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream);
/* Diagnostic (tools/trace_persist.py --config cfg3): one persistent SCAMP forward with s_memtime
 * stamps per (workgroup, iteration, phase) into `trace` (ceil(B/16) * max_iter * 10 uint64). */
int amp_scamp_persist_trace(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* trace,
                            void* stream);
/* SCAMP.forward + Loss.error_rate in one call (scamp.py:77-107 then loss.py:67-179), as
 * amp_vamp_detect_count: the persistent engine's forward with the MAP decision on xmap
 * (scamp.py:107) fused into the same launch (each workgroup decides the rows it holds in LDS; one
 * fold launch after it), counters identical to amp_map_decide_count's.  AMP_E_ARG when the shape
 * is not persistent-eligible (use amp_scamp_run + amp_map_decide_count). */
int amp_scamp_detect_count(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a,
                           const amp_vamp_decide_args* dec, void* stream);
/* amp_scamp_run (launch engine) on one rank's slice of a trial-sharded batch (the protocol of
 * amp_vamp_run_sharded, the hook of amp_set_allreduce_hook): max|xi| / min section max
 * (scamp.py:64), the psi allclose count (scamp.py:105) and the rare path's exact values
 * all-reduced per iteration; decision on xmap with amp_map_decide_count_rows. */
int amp_scamp_run_sharded(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a,
                          int32_t B_global, void* stream);
/* Layer-level pieces of amp_scamp_run, as for BAMP: prepare = Tracker (scamp.py:9-25), iterate(t)
 * = one SCAMPLayer.forward (scamp.py:43-59) + the allclose(psi) early exit of scamp.py:105,
 * finalize = the last psi into a->psi. */
int amp_scamp_prepare(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream);
int amp_scamp_iterate(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, int32_t t,
                      void* stream);
int amp_scamp_finalize(const amp_dims* d, const amp_constellation* c, const amp_scamp_args* a, void* stream);

/* ---- Block-sparse denoiser — replaces VAMPLayer.segmented_denoiser
 *      (vamp.py:96-119), BAMPLayer.segmented_denoiser (bamp.py:66-77) and
 *      SCAMPLayer.denoiser (scamp.py:61-68) as a standalone op.
 * tau_mode 0: tau = tau_scalar (VAMP sigma2); 1: tau[b][j] = tau_vec[b*N+j]*0.5 (BAMP cov);
 *          2: as 1 but mean only (SCAMP, var may be NULL).
 * The batch-global float64 max|xi| shift of the reference is reproduced by its
 * NaN rule: a section is NaN iff its max logit lies > 745.1332 below max|xi|. */
int amp_block_denoise(const amp_dims* d, const amp_constellation* c, const void* r, int32_t tau_mode,
                      float tau_scalar, const void* tau_vec, void* xmmse, void* var, void* ws,
                      size_t ws_bytes, void* stream);
size_t amp_block_denoise_workspace_bytes(const amp_dims* d);

/* ---- MAP decision + error counting — replaces Loss.error_rate (loss.py:67-103),
 *      Loss.MAP_decision (loss.py:282-302) and the metric helpers (loss.py:105-179).
 * sym: int64 [B*L] true gray labels; idx: int64 [B*L] true flat nonzero indices
 * (data.py:89-90).  ibits_trunc = ceil(log2(Lin*B*Na)) (loss.py:20).
 * decisions (optional, may be NULL): int32 [B*L] flat argmax m*K + k per section. */
int amp_map_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap,
                         const void* xmmse, const void* x, const void* sym, const void* idx,
                         int32_t ibits_trunc, void* counts, void* decisions, void* ws, size_t ws_bytes,
                         void* stream);
/* The same over rows [row0, row0 + d->B) of a larger batch (a trial-sharded rank's slice): the
 * flat indices it compares (loss.py:105-169) are those of the whole batch, so the chosen entry's
 * flat index is formed at section (row0 + b) * L + l; sym / idx hold this slice's labels.  The
 * ranks' counters sum to the whole batch's. */
int amp_map_decide_count_rows(const amp_dims* d, const amp_constellation* c, const void* xmap,
                              const void* xmmse, const void* x, const void* sym, const void* idx,
                              int32_t ibits_trunc, int64_t row0, void* counts, void* decisions, void* ws,
                              size_t ws_bytes, void* stream);
size_t amp_map_decide_workspace_bytes(const amp_dims* d);
/* Same counters with Loss.random_decision (loss.py:252-280, generator_mode='random'): per
 * channel use the Na largest |x_m| (NaN largest; exact ties by larger index), each decided to
 * its nearest point, compared in ascending position order with the row's true sorted indices.
 * decisions (optional): int32 [B*Lin*Na], position * K + k.  Na <= 64.  Same workspace. */
int amp_random_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap,
                            const void* xmmse, const void* x, const void* sym, const void* idx,
                            int32_t ibits_trunc, void* counts, void* decisions, void* ws,
                            size_t ws_bytes, void* stream);
/* Same counters with Loss.segmented_decision (loss.py:222-250, generator_mode='segmented'):
 * per section the largest |x_m| (last index on ties, NaN largest), then the nearest point
 * |x_m - a_k| (first minimum).  The reference only runs it for B = 1 (its reshape drops the
 * batch axis); this entry point takes any B.  Same arguments and workspace as above. */
int amp_segmented_decide_count(const amp_dims* d, const amp_constellation* c, const void* xmap,
                               const void* xmmse, const void* x, const void* sym, const void* idx,
                               int32_t ibits_trunc, void* counts, void* decisions, void* ws,
                               size_t ws_bytes, void* stream);

/* ---- Element-wise shrinkage denoisers — replace Shrink (shrink.py:8-166).
 * r: [count] complex64 (is_complex != 0) or float32; cov: cov_vec [count] float32, or
 * cov_scalar when cov_vec is NULL (a 0-dim tensor in the reference).
 * amp_shrink_bayes   Shrink.bayes (shrink.py:78-96): out [count], same dtype as r;
 *                    P0, Ps = Config.P0 / Config.Ps as float32 (shrink.py:19).
 * amp_shrink_ook     Shrink.shrinkOOK (shrink.py:139-157): exp_out [count] float32 and
 *                    dxdr_out = one float32, der.mean() over all count elements;
 *                    theta = float32 log(P0/Ps) (shrink.py:152).  count must be > 0.
 * amp_shrink_sw_ook  Shrink.sw_shrinkOOK (shrink.py:58-76) over `sections` sections of M:
 *                    exp_out [sections*M] complex64 (imaginary 0), var_out float32.
 * Shrink.shrink / Shrink.lasso (shrink.py:98-137) raise for every input in the reference
 * and have no entry point. */
int amp_shrink_bayes(const amp_constellation* c, int64_t count, int32_t is_complex, const void* r, float cov_scalar,
                     const void* cov_vec, float P0, float Ps, void* out, void* stream);
int amp_shrink_ook(int64_t count, int32_t is_complex, const void* r, float cov_scalar, const void* cov_vec,
                   float theta, void* exp_out, void* dxdr_out, void* ws, size_t ws_bytes, void* stream);
size_t amp_shrink_ook_workspace_bytes(int64_t count);
int amp_shrink_sw_ook(int64_t sections, int32_t M, int32_t is_complex, const void* r, float cov_scalar,
                      const void* cov_vec, void* exp_out, void* var_out, void* stream);

/* ---- Building blocks exposed for tests and tools ---- */
/* C[rows][ldc] = A[rows][lda] . Wt[ncp][kap]^T on fp32 MFMA (first ka columns of A, first nc of C);
   Wt row-major, kap % 64 == 0, ncp % 128 == 0, lda % 4 == 0. */
int amp_gemm_nt_f32(const void* a, int32_t lda, int32_t rows, int32_t ka, const void* wt, int32_t kap,
                    int32_t ncp, void* c, int32_t ldc, int32_t nc, void* stream);
/* Real expansion of a complex operator X[o][j] = rowscale[o] * op(src[o*so + j*sj]) into Wt. */
int amp_build_cweight(const void* src, int64_t so, int64_t sj, int32_t conj, const void* rowscale,
                      int32_t O, int32_t J, void* wt, int32_t kap, int32_t ncp, void* stream);

/* ---- damped "Rangan" VAMP — replaces vamp2.py's VAMP.forward (vamp2.py:103-135), Tracker
 *      (:12-26) and VAMPLayer.forward (:52-77) with its segmented denoiser (:79-88).  The
 *      reference's VAMP passes damping = 1.0 (vamp2.py:96); sparc mode only (the reference crashes
 *      in 'random' / 'segmented' mode).  status.last_scalar = {gamma, alpha, gamma~, d.mean()}. */
typedef struct amp_vamp2_args {
    const void* U;      /* c64 [n][k] */
    const void* s;      /* f32 [k] */
    const void* Vh;     /* c64 [k][N] */
    const void* y;      /* c64 [B][n] */
    int32_t k;          /* min(n, N) */
    int32_t max_iter;   /* config.N_Layers */
    double sigma2;      /* Na/Nr/SNR (vamp2.py:123, Python float) */
    double damping;     /* rho (vamp2.py:50) */
    void* r;            /* out c64 [B][N]: T.r, the decision input (vamp2.py:131) */
    void* xmmse;        /* out c64 [B][N]: the damped T.xmmse */
    void* var;          /* out f32 [B][N] */
    void* status;       /* out amp_status (device) */
    void* ws;           /* workspace, amp_vamp2_workspace_bytes() bytes */
    size_t ws_bytes;
} amp_vamp2_args;
size_t amp_vamp2_workspace_bytes(const amp_dims* d, int32_t k);
int amp_vamp2_run(const amp_dims* d, const amp_constellation* c, const amp_vamp2_args* a, void* stream);

/* A stream whose kernels run only on CUs [cu0, cu1) of the current device (its own hardware queue):
 * the co-resident grids of amp_vamp_detect_count_shard on one GPU, each on its own CUs. */
int amp_stream_create_cu_range(int32_t cu0, int32_t cu1, void** stream);
int amp_stream_destroy(void* stream);

/* Diagnostics. */
const char* amp_last_error(void);
const char* amp_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* AMP_SPARC_H */

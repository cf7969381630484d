/*
 * dfq_hip.h -- C ABI of libdfq_hip.so, the MI355X (gfx950) data-free-quantization
 * weight-transform path.
 *
 * Every entry point is plain C: raw device pointers, integer sizes, an opaque
 * hipStream_t passed as `void*` (NULL = the legacy default stream).  All compute
 * calls are asynchronous on that stream unless the comment says "blocking".
 * Nothing here allocates device memory on the hot path: the one-shot calls take
 * a caller-provided workspace, and the plan objects allocate once at create().
 *
 * Return value: 0 on success, a negative DFQ_ERR_* code otherwise
 * (dfq_error_string() gives the text).  The Python host layer maps
 * DFQ_ERR_SHAPE to ValueError/RuntimeError exactly where the reference raises.
 *
 * Each function cites the reference interface (KadAMRN/Data_Free_Quantization)
 * whose arithmetic it replaces.  The binding a maintainer adds on the reference
 * side (ctypes) is in INTEGRATION.md.
 */
#ifndef DFQ_HIP_H_
#define DFQ_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* The library is built with hidden visibility: only these entry points are
 * exported (two builds in one process -- the product and the diagnostics
 * library -- then never bind to each other's internals). */
#pragma GCC visibility push(default)

#define DFQ_ABI_VERSION 1

/* Load every kernel's code object on the current device now (otherwise the first
 * launch from each translation unit pays for it, ~ms), and allocate what a first
 * run would allocate inside the caller's timing: the CLE context's stream, table
 * pools (4 MB device, 2 MB pinned), iteration history, signal word and worker
 * thread, and 8 pinned 1 MB staging slots for table uploads.  main_dfq calls it
 * (`_lib.preload()`) before its timer, as process setup.  Idempotent, blocking;
 * 0 or DFQ_ERR_HIP. */
int dfq_preload(void);

/* ---- error codes ------------------------------------------------------- */
#define DFQ_OK              0
#define DFQ_ERR_INVALID    -1   /* bad argument (null pointer, bits out of range, ...) */
#define DFQ_ERR_HIP        -2   /* a HIP runtime call failed */
#define DFQ_ERR_UNSUPPORTED -3  /* valid request this build does not implement */
#define DFQ_ERR_NOMEM      -4   /* device / host allocation failed (plan create only) */
#define DFQ_ERR_SHAPE      -5   /* shape mismatch the reference would raise on */
#define DFQ_ERR_WORKSPACE  -6   /* caller workspace too small */

/* ---- quantizer modes ---------------------------------------------------- */
/* TENSOR_* use one (min, max) for the whole tensor (reference default,
 * utils/quantize.py:62-66 via utils/layer_transform.py:298).  CHANNEL_* use one
 * (min, max) per row = per output channel (extension: the reference quantize()
 * applied to each W[o] slice).  *_SYM is utils/quantize.py:51-60.              */
#define DFQ_TENSOR_ASYM   0
#define DFQ_TENSOR_SYM    1
#define DFQ_CHANNEL_ASYM  2
#define DFQ_CHANNEL_SYM   3

/* ---- descriptor flags --------------------------------------------------- */
#define DFQ_CLIP          0x1  /* clamp the dequantized output to [clip_lo, clip_hi] (clip_weight.py:29) */
#define DFQ_GIVEN_RANGE   0x2  /* use given_min/given_max (Python doubles) instead of the data range */
#define DFQ_SCALE_F32     0x4  /* scale arithmetic in fp32 (quantize() called with min/max=None,
                                  utils/quantize.py:26-37: 0-d fp32 tensors) instead of fp64;
                                  with DFQ_GIVEN_RANGE the given values are fp32 tensor values */
#define DFQ_PACK_INT4     0x8  /* bits <= 4: codes packed two per byte, element 2k in the low nibble and
                                  2k+1 in the high nibble (two's-complement nibbles when symmetric);
                                  codes holds ceil(rows*row_len/2) bytes.  bits > 4: DFQ_ERR_INVALID.
                                  Every task starts at an even element, so per channel an odd row_len
                                  above half a task (1024 elements by default) with rows > 1 is
                                  DFQ_ERR_UNSUPPORTED (two rows' tasks would share a byte) */

#define DFQ_DEVICE_RANGE  0x10 /* TENSOR modes: the range is read on the device, when the sweep runs,
                                  from range_enc = {~enc(min), enc(max)} (dfq_range's encoding, or
                                  the by-product of dfq_bn_fold_batch): one HBM pass, no reduce
                                  launch.  Arithmetic as for the data range (the values are the
                                  tensor's fp32 min and max).  Not with DFQ_GIVEN_RANGE */

/* One fp32 tensor viewed as [rows, row_len], row_len = I*KH*KW (KCRS) or I (Linear).
 * Outputs are written only where the pointer is non-NULL:
 *   dst    fp32 dequantized values (may alias src: in-place, like weight.data.copy_)
 *   codes  integer grid indices: uint8 (asym, bits<=8), int8 (sym, bits<=8),
 *          uint16/int16 for 8<bits<=16, or packed nibbles (DFQ_PACK_INT4)
 *   scale  fp32 step, [rows] in CHANNEL modes, [1] in TENSOR modes
 *   zero   fp32 value added back after scaling (the range min for asym, +0 for sym)
 *   esum   fp32 bias-correction error sums E[o,i] = sum_k (y - x)[o, i*khw + k],
 *          [rows * row_len/khw]  (bias_correction.py:128-131,231 on the fused output y)
 */
typedef struct dfq_tensor_desc {
    const float* src;
    float*       dst;
    void*        codes;
    float*       scale;
    float*       zero;
    float*       esum;
    int64_t      rows;
    int64_t      row_len;
    int32_t      khw;       /* spatial size for esum (1 for Linear / 1x1) */
    int32_t      bits;      /* 2..16 */
    int32_t      mode;      /* DFQ_TENSOR_ASYM ... DFQ_CHANNEL_SYM */
    int32_t      flags;     /* DFQ_CLIP | DFQ_GIVEN_RANGE | DFQ_SCALE_F32 | DFQ_PACK_INT4 | DFQ_DEVICE_RANGE */
    float        clip_lo;
    float        clip_hi;
    double       given_min;
    double       given_max;
    const uint32_t* range_enc; /* DFQ_DEVICE_RANGE: 2 device words, else NULL */
} dfq_tensor_desc;

/* ---- library ------------------------------------------------------------ */
int         dfq_abi_version(void);
const char* dfq_error_string(int code);
/* Last HIP error text seen by the library on this thread ("" if none). */
const char* dfq_last_hip_error(void);

/* ---- single-tensor quantize (replaces quantize()/UniformQuantize.forward,
 *      utils/quantize.py:16-89) ------------------------------------------- */
/* Workspace bytes dfq_quantize_tensor needs for this descriptor (0 is possible). */
int dfq_quantize_ws_bytes(const dfq_tensor_desc* desc, size_t* bytes);
/* Asynchronous on `stream` (the task table goes up through the library's pinned
 * staging ring; no host wait).  ws: device memory of >= dfq_quantize_ws_bytes
 * bytes that stays allocated until the stream reaches the kernel (a
 * stream-ordered allocator does that). */
int dfq_quantize_tensor(const dfq_tensor_desc* desc, void* ws, size_t ws_bytes, void* stream);
/* quantize()'s data range when min/max are None and num_chunks splits the batch
 * (utils/quantize.py:26-37): x viewed as [rows = B // num_chunks, row_len];
 * out2 = {mean_r min(x[r]), mean_r max(x[r])} in fp32, the mean in ATen's sum
 * order.  rowbuf: 2*rows device floats of scratch.  Async on `stream`. */
int dfq_chunk_range(const float* x, int64_t rows, int64_t row_len, float* rowbuf, float* out2, void* stream);
/* QuantMeasure.forward's statistics (utils/quantize.py:94-126), async, two
 * launches: mn / mx = the means over rows of x.view(rows, -1)'s row mins / maxs
 * (fp32, ATen's sum order); update_stat: running_max = mx if mx > running_max
 * (running_min likewise); training: running_* = running_* * (1 - momentum) +
 * (mn|mx) * momentum (fp32 ops, in that order, after the update).  out2 (2 device
 * floats) = the range the fake quant then uses: (mn, mx) in training, the running
 * values otherwise.  words: 2*rows device uint32 of per-observer scratch, zeroed
 * ONCE by the caller; every call leaves them zeroed again.  Replaces the
 * QuantMeasure statistics of the reference (no C counterpart there). */
int dfq_act_observe(const float* x, int64_t rows, int64_t row_len, uint32_t* words, float* running_min,
                    float* running_max, int32_t update_stat, int32_t training, double momentum, float* out2,
                    void* stream);
/* Whole-tensor (min, max) on the device, async: range_enc (2 device uint32) =
 * {~enc(min), enc(max)} in the library's order-preserving encoding (the input of
 * dfq_fake_quant_given); it is zeroed on `stream` first. */
int dfq_range(const float* x, int64_t n, uint32_t* range_enc, void* stream);
/* quantize(x, bits, min, max, symmetric) with a GIVEN range, elementwise and async
 * (QuantMeasure.forward at inference, utils/quantize.py:112-126, and the Quant*
 * layers' weight/bias fake quant, :225-238): the range is, by priority,
 * range_enc (dfq_range's output), min_dev[0] / max_dev[0] (device floats, e.g. the
 * observer's running_min / running_max, read as float() would: exact doubles), or
 * given_min / given_max.  flags: 0 (scale in double: Python-float bounds) or
 * DFQ_SCALE_F32 (0-d tensor bounds).  No workspace, no host synchronisation. */
int dfq_fake_quant_given(const float* x, float* y, int64_t n, int32_t bits, int32_t symmetric, int32_t flags,
                         const float* min_dev, const float* max_dev, const uint32_t* range_enc, double given_min,
                         double given_max, void* stream);

/* quantize(x, bits, float(x.min()), float(x.max()), symmetric) -- the Quant* layers'
 * weight / bias fake quant (utils/quantize.py:225-238) on the tensor's own range --
 * in one async call: dfq_range + dfq_fake_quant_given without the fill.  n <= 16384:
 * one workgroup, one launch (words may be NULL); larger: a range launch whose last
 * block publishes the range and re-arms `words`, then the elementwise launch.
 * words: 8 device uint32 of caller scratch, zero when allocated, left armed by every
 * call (one set per stream: calls on two streams must not share it).  flags: 0 or
 * DFQ_SCALE_F32, as dfq_fake_quant_given. */
int dfq_fake_quant_tensor(const float* x, float* y, int64_t n, int32_t bits, int32_t symmetric, int32_t flags,
                          uint32_t* words, void* stream);

/* ---- grouped sweep over many tensors (replaces quantize_targ_layer,
 *      utils/layer_transform.py:288-305, fused with clip_weight.py:4-33 and the
 *      bias-correction error reduction bias_correction.py:111-144,231) ------- */
typedef struct dfq_sweep_plan dfq_sweep_plan;
typedef struct dfq_sweep_stats {
    int64_t n_tensors;
    int64_t n_elems;          /* sum of rows*row_len */
    int64_t n_tasks_reduce;   /* wave tasks of the range-reduction launch (0 = launch skipped) */
    int64_t n_tasks_main;     /* wave tasks of the quantize launch */
    int64_t algo_bytes;       /* algorithmic HBM bytes of one execute */
    int32_t launches;         /* kernel launches per execute (1, or 2 with a reduce pass) */
    int32_t grid_blocks;      /* blocks of the quantize launch */
    int32_t variant;          /* kernel variant (env DFQ_SWEEP_VARIANT at create) */
    int32_t reserved;
} dfq_sweep_stats;
/* Uploads the descriptor/task tables once into a private allocation (a blocking
 * copy).  descs is copied. */
int dfq_sweep_plan_create(const dfq_tensor_desc* descs, int32_t n, dfq_sweep_plan** plan);
/* The same with the tables in a caller workspace of >= dfq_sweep_plan_ws_bytes
 * bytes (256-B aligned, stream-ordered with `stream`, alive while the plan runs;
 * e.g. the framework's caching allocator): no hipMalloc / hipFree, and destroy
 * needs no device sync.  The upload is stream-ordered on `stream` (pinned
 * staging ring, no host wait). */
int64_t dfq_sweep_plan_ws_bytes(const dfq_tensor_desc* descs, int32_t n);
int dfq_sweep_plan_create_ws(const dfq_tensor_desc* descs, int32_t n, void* ws, int64_t ws_bytes, void* stream,
                             dfq_sweep_plan** plan);
int dfq_sweep_plan_execute(dfq_sweep_plan* plan, void* stream);
int dfq_sweep_plan_stats(const dfq_sweep_plan* plan, dfq_sweep_stats* stats);
int dfq_sweep_plan_destroy(dfq_sweep_plan* plan);

/* ---- BatchNorm folding (merge_batchnorm, utils/layer_transform.py:255-281) ---
 * w[o,:] *= g[o]/sqrt(v[o]+eps);  bias[o] = bias[o]*f[o] + (b[o] - g[o]*m[o]/sqrt(v[o]+eps));
 * fake_w = |g|, fake_b = b (either may be NULL); then the BN becomes identity:
 * g=1, v=1, b=0, m=0 (the caller sets module.eps = 0).  rows = O, row_len = numel/O. */
int dfq_bn_fold(float* w, float* bias, float* bn_w, float* bn_b, float* bn_mean, float* bn_var,
                float* fake_w, float* fake_b, float eps, int64_t rows, int64_t row_len,
                void* stream);

/* All BN folds of a model in two launches: one descriptor per (BN, producer
 * layer) pair, each weight at most once per call; eps per BN.  Stream-ordered
 * with a workspace, blocking without one (see ws below). */
enum { DFQ_BN_FOLD_ZERO_BIAS = 1 };
typedef struct dfq_bn_fold_desc {
    float* w;
    float* bias;
    float* bn_w;
    float* bn_b;
    float* bn_mean;
    float* bn_var;
    float* fake_w;      /* may be NULL */
    float* fake_b;      /* may be NULL */
    float  eps;
    int32_t flags;      /* DFQ_BN_FOLD_ZERO_BIAS: `bias` holds no value yet and is read as 0
                         * (the zeros the reference gives a bias-less layer) */
    int64_t rows;
    int64_t row_len;
    uint32_t* range_enc; /* may be NULL: 2 device words receiving the folded weight's (min, max) in
                          * dfq_range's encoding (zeroed by the call), for a later sweep with
                          * DFQ_DEVICE_RANGE.  Rows whose factor is exactly 1 (merge_batchnorm #2)
                          * are read, not rewritten (w * 1 == w) */
} dfq_bn_fold_desc;
/* Device workspace bytes for dfq_bn_fold_batch's job tables (-1: bad arguments). */
int64_t dfq_bn_fold_ws_bytes(const dfq_bn_fold_desc* descs, int32_t n);
/* ws: >= dfq_bn_fold_ws_bytes bytes, 256-B aligned, stream-ordered with `stream`
 * (e.g. the framework's caching allocator), or NULL: private tables (a
 * hipMalloc / hipFree per call).  With ws the call is stream-ordered (tables go
 * up through the library's pinned staging ring; no host wait); with NULL it
 * synchronizes the stream before freeing its private tables. */
int dfq_bn_fold_batch(const dfq_bn_fold_desc* descs, int32_t n, void* ws, int64_t ws_bytes, void* stream);

/* ---- weight clipping (clip_weight.py:18-29): w = min(max(w, lo), hi), in place */
int dfq_clamp(float* w, int64_t n, float lo, float hi, void* stream);
/* clip_weight over every target layer: `count` weights (16-B aligned, w[k] of
 * n[k] floats), up to 64 per launch. */
int dfq_clamp_batch(float* const* w, const int64_t* n, int32_t count, float lo, float hi, void* stream);

/* ---- cross-layer equalization (Cross_layer_equal.py) -------------------- */
/* Workspace bytes for one relation with c1 = W1.shape[0] channels. */
size_t dfq_cle_ws_bytes(int64_t c1);
/* One relation (_layer_equalization, Cross_layer_equal.py:11-59), in place:
 *   W1 [c1, len1] rows, W2 [o2, i2, khw2], B1/bn_w/bn_b [c1] (each may be NULL),
 *   groups G = (c1 == i2) ? 1 : c1 / i2.
 * S (may be NULL) receives the per-channel scale; S_acc (may be NULL) is
 * multiplied by it (Relation.set_scale_vec, utils/relation.py:26-30; pass
 * s_acc_init=1 on the first call to store instead of multiply). */
int dfq_cle_relation(float* w1, float* w2, float* b1, float* bn_w, float* bn_b,
                     int64_t c1, int64_t len1, int64_t o2, int64_t i2, int64_t khw2,
                     double s_min, double s_max, int32_t is_signed, float eps,
                     float* S, float* S_acc, int32_t s_acc_init,
                     void* ws, size_t ws_bytes, void* stream);
/* Convergence metric of Cross_layer_equal.py:83,107-108 for a set of layers:
 * out_mean[l] = (double)(float)( sum|W_l - snap_l| / n_l ), then snap_l := W_l.
 * Blocking: waits for the stream and copies the n means to host memory. */
typedef struct dfq_diff_plan dfq_diff_plan;
int dfq_diff_plan_create(float* const* w, float* const* snap, const int64_t* n, int32_t count,
                         dfq_diff_plan** plan);
int dfq_diff_plan_snapshot(dfq_diff_plan* plan, void* stream);  /* snap := W, async */
int dfq_diff_plan_execute(dfq_diff_plan* plan, double* out_mean, void* stream);
int dfq_diff_plan_destroy(dfq_diff_plan* plan);

/* Device-resident cross_layer_equalization loop (Cross_layer_equal.py:63-116).
 * One relation of the loop (:86-104); pointers are device memory, in place. */
typedef struct dfq_cle_rel {
    float* w1;          /* graph[layer_first].weight, [c1, len1] */
    float* w2;          /* graph[layer_second].weight, [o2, i2, khw2] */
    float* b1;          /* graph[layer_first].bias [c1] (the caller adds the zero bias of :93-94) */
    float* bn_w;        /* graph[bn_idx].fake_weight [c1] or NULL */
    float* bn_b;        /* graph[bn_idx].fake_bias [c1] or NULL */
    float* s_acc;       /* Relation.S [c1] (set_scale_vec, utils/relation.py:26-30) or NULL */
    int64_t c1, len1, o2, i2, khw2;
    int32_t s_acc_init; /* Relation.S was None: the first iteration stores s */
    int32_t reserved;
} dfq_cle_rel;
typedef struct dfq_cle_plan dfq_cle_plan;
/* Workspace bytes for the plan's weight snapshots (the `W_prev` of :83,107):
 * one fp32 copy of every target, each 256-B aligned; -1 on bad arguments. */
int64_t dfq_cle_plan_ws_bytes(const int64_t* target_n, int32_t n_targets);
/* targets: the weights of every Target_list layer in graph order (the diff list of
 * :107); ref_threads: torch's intra-op thread count whose fp32 mean order the
 * metric reproduces. Relations touching a common tensor keep their order; the
 * others run concurrently (bit-identical: they commute).
 * ws: caller-owned device workspace of >= dfq_cle_plan_ws_bytes bytes, 256-B
 * aligned, alive until destroy (e.g. from the framework's caching allocator), or
 * NULL: the plan allocates it. */
int dfq_cle_plan_create(const dfq_cle_rel* rels, int32_t n_rel, float* const* targets,
                        const int64_t* target_n, int32_t n_targets, double s_min, double s_max,
                        int32_t is_signed, float eps, int32_t ref_threads, void* ws, int64_t ws_bytes,
                        dfq_cle_plan** plan);
/* Runs the loop `while diff > threshold and iter_count < count` (at most
 * max_iters iterations); blocking.  iterations = iterations run; diffs[i] (room for
 * max_iters doubles, may be NULL) = the per-iteration diff (np.sum of the list). */
int dfq_cle_plan_run(dfq_cle_plan* plan, double threshold, int32_t count, int32_t max_iters,
                     int32_t* iterations, double* diffs, void* stream);
/* The same loop, asynchronous (a worker thread reads the stop rule back between
 * batches): `stream`'s earlier work runs before the loop, and everything enqueued
 * on `stream` after this call waits in the device until the loop is done -- the
 * caller's thread goes on enqueueing the next stages meanwhile (the caller's
 * stream waits behind a one-wave gate kernel that polls the library's signal
 * word; it gives up after 120 s, and the join then reports the run failed).
 * A launched run is time-bounded: it stops enqueueing iterations 60 s after the
 * launch, releases the caller's stream and reports the run failed at join (the
 * stages queued behind it then ran on partially equalized weights, so the join's
 * error must not be ignored); a blocking run (dfq_cle_plan_run) has no time
 * bound and stops at max_iters.
 * One launched plan per device at a time (a launch first joins the previous one).
 * DFQ_ERR_UNSUPPORTED: the device cannot make a stream wait on a value (run
 * dfq_cle_plan_run instead). */
int dfq_cle_plan_launch(dfq_cle_plan* plan, double threshold, int32_t count, int32_t max_iters, void* stream);
/* Waits for a launched run; its result as dfq_cle_plan_run's (diffs: room for
 * max_iters doubles, may be NULL).  destroy also waits. */
int dfq_cle_plan_join(dfq_cle_plan* plan, int32_t* iterations, double* diffs);
/* chains = independent relation groups, steps = relations per chain (max),
 * launches = kernel launches per iteration (fused schedule: one range launch for
 * the whole iteration; DFQ_CLE_FUSED=0: one per step) */
int dfq_cle_plan_info(const dfq_cle_plan* plan, int32_t* chains, int32_t* steps, int32_t* launches);
/* Measurement (no reference counterpart): with timing on, the next run records one
 * HIP event pair on the loop's stream around its launches.  stats: bytes[3] = the
 * algorithmic HBM bytes of ONE iteration (rescales incl. the per-channel vectors,
 * metric tiles, weight-reading range tasks), loop_ms = the last timed run's device
 * time from its first launch to its last (-1 if not timed), launched = the
 * iteration groups it enqueued (iterations + the queued no-op ones). */
int dfq_cle_plan_set_timing(dfq_cle_plan* plan, int32_t on);
int dfq_cle_plan_stats(const dfq_cle_plan* plan, int64_t* bytes, double* loop_ms, int32_t* launched);
int dfq_cle_plan_destroy(dfq_cle_plan* plan);

/* ---- high-bias absorption (bias_absorption.py:147-197) ------------------
 * c = max(bn_b - N*bn_w, 0) (bn_* = the BN's fake_weight / fake_bias);
 * b2[o] += sum_i (sum_k W2[o,i,k]) * c[g*i2 + i];  b1 -= c;  bn_b -= c.
 * W2 is [o2, i2, khw2], c1 = W1.shape[0], groups = c1 / i2. */
int dfq_bias_absorb(const float* w2, float* b1, float* b2, float* bn_w, float* bn_b,
                    int64_t c1, int64_t o2, int64_t i2, int64_t khw2, float n_sigma,
                    void* stream);
/* Every absorption of a model in two launches (bias_absorption.py:9-121, the
 * relations in the reference's order): all c = clamp(beta - N*gamma, 0) and
 * W2-sum GEMVs first (into the workspace), then one pass per bias element that
 * applies that vector's updates in relation order (b -= c as a layer_first,
 * b += W2sum @ c as a layer_second) and beta -= c -- the same fp32 operations in
 * the same per-element order as one dfq_bias_absorb call per relation.
 * `*failed` = the index of a relation whose shapes are invalid (nothing is
 * enqueued then). */
typedef struct dfq_absorb_desc {
    const float* w2;
    float*       b1;
    float*       b2;
    float*       bn_w;    /* fake_weight of the BN between the layers */
    float*       bn_b;    /* fake_bias (updated) */
    int64_t      c1, o2, i2, khw2;
} dfq_absorb_desc;
int64_t dfq_bias_absorb_ws_bytes(const dfq_absorb_desc* descs, int32_t n);
int dfq_bias_absorb_batch(const dfq_absorb_desc* descs, int32_t n, float n_sigma, void* ws, int64_t ws_bytes,
                          int32_t* failed, void* stream);

/* ---- bias correction (bias_correction.py) -------------------------------
 * dfq_bc_expect: out[j] (+)= relu ? max(0, w*phi(-b/w) + b*(1-Phi(-b/w))) : b
 *                (calculate_mean + branch sum, bias_correction.py:33-53,170-172). */
int dfq_bc_expect(const float* fake_w, const float* fake_b, int64_t n, int32_t relu,
                  int32_t accumulate, float* out, void* stream);
/* dfq_bc_apply: bias_vec[o,j] = E[o, i2>1 ? j : 0] + expect[f>1 ? j : 0] over the
 * broadcast shape [o, bcols]; bias[o] += mean_j bias_vec[o,j] (ATen's sum order)
 * (_compute_final_bias_correction + _apply_bias_correction, :61-106).
 * bias_vec (may be NULL) keeps the [o*bcols] vector for dfq_bc_propagate.
 * Returns DFQ_ERR_SHAPE where torch would raise (non-broadcastable, or numel == o). */
int dfq_bc_apply(const float* E, int64_t o, int64_t i2, const float* expect, int64_t f,
                 float* bias, float* bias_vec, int64_t* bcols_out, void* stream);
/* dfq_bc_propagate: fake_b[c] += mean_r ( -bias_vec[r*f + c] ), r < numel/f
 * (bias_prev.view(-1, F).mean(0), bias_correction.py:206-213,251).  The fp32 sums
 * follow ATen's CPU reduction order for `ref_threads` intra-op threads (the
 * reference's torch.get_num_threads()). */
int dfq_bc_propagate(const float* bias_vec, int64_t numel, float* fake_b, int64_t f,
                     int32_t ref_threads, void* stream);

/* dfq_bc_chain: a whole bias_correction walk's device work in one call -- the
 * ops above, recorded by the host walk in graph order and enqueued back to back
 * on `stream` (bias_correction.py:147-258 issues them one Python call each).
 * COPY ops (the walk's before/after bias snapshots, bias_correction.py:196,255)
 * copy n floats; consecutive ones share a launch.
 * Every op is validated before the first launch; a bad op returns its error code
 * and `*failed_op` = its index, with nothing enqueued. */
enum { DFQ_BC_OP_EXPECT = 0, DFQ_BC_OP_APPLY = 1, DFQ_BC_OP_PROPAGATE = 2, DFQ_BC_OP_COPY = 3 };
/* APPLY flag: out2 (bias_vec) is chain scratch -- only this chain's ops read it,
 * and its contents after the call are unspecified, so the one-launch path may
 * leave it unwritten where every reader recomputes it (the Python walk's vectors). */
enum { DFQ_BC_APPLY_VEC_SCRATCH = 1 };
typedef struct dfq_bc_op {
    int32_t      kind;      /* DFQ_BC_OP_* */
    int32_t      flag;      /* EXPECT: relu | (accumulate << 1); APPLY: DFQ_BC_APPLY_VEC_SCRATCH or 0;
                               PROPAGATE: ref_threads */
    const float* a;         /* EXPECT: fake_w  APPLY: E       PROPAGATE: bias_vec  COPY: src */
    const float* b;         /* EXPECT: fake_b  APPLY: expect */
    float*       out;       /* EXPECT: out     APPLY: bias    PROPAGATE: fake_b    COPY: dst */
    float*       out2;      /* APPLY: bias_vec (may be NULL) */
    int64_t      n;         /* EXPECT: n       APPLY: o       PROPAGATE: numel     COPY: floats */
    int64_t      i2;        /* APPLY: i2 */
    int64_t      f;         /* APPLY: expect numel  PROPAGATE: F */
} dfq_bc_op;
int dfq_bc_chain(const dfq_bc_op* ops, int32_t n_ops, int32_t* failed_op, void* stream);

/* ---- activation ranges from BN statistics (set_quant_minmax,
 *      utils/layer_transform.py:356-618) ---------------------------------------
 * Per channel j, with w = sqrt_w ? sqrt(w[j] + eps) : w[j], b = b[j]:
 *   kind 0: m = b, v = w*w;  1: calculate_mean / calculate_var (ReLU, :396-399);
 *   2: calculate_mean_6 / calculate_var_6 (ReLU6, :400-410);
 *   accumulate ? (mean += m, var += v) : (mean = m, var = v).  mean/var may alias w/b. */
int dfq_act_moments(const float* w, const float* b, int64_t n, int32_t kind, int32_t sqrt_w, float eps,
                    int32_t accumulate, float* mean, float* var, void* stream);
/* out2 = {min(a - nsig*w), max(a + nsig*w)} (get_min_value / get_max_value, :391-392),
 * w := sqrt(w + eps) when w_is_var.  out2: 2 device floats. */
int dfq_act_minmax(const float* a, const float* w, int64_t n, int32_t w_is_var, float eps, float nsig,
                   float* out2, void* stream);
/* Case (d.) (:470-481): out[o] = sum_i (sum_k W[o,i,k]) * x[g*i2 + i] (+ bias[o]),
 * W = [o, i2, khw] (khw = 1 for Linear), g = o / (o / groups). */
int dfq_act_affine(const float* x, const float* w, const float* bias, int64_t o, int64_t i2, int64_t khw,
                   int64_t groups, float* out, void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* DFQ_HIP_H_ */

/*
 * dfq_diag.h -- diagnostics entry points of libdfq_diag.so (NOT the product).
 *
 * libdfq_diag.so is the product library (every dfq_hip.h entry point) built with
 * -DDFQ_DIAGNOSTICS: it also carries the sweep's A/B kernel variants and
 * environment switches (DFQ_SWEEP_VARIANT, DFQ_CLE_FUSED, DFQ_CLE_TILES_EARLY, ...)
 * and the probes below, which bench.py and scripts/ use to measure the ceiling
 * of the sweep's memory pattern.  None of this is part of the reference
 * interface; libdfq_hip.so exports none of it.
 */
#ifndef DFQ_DIAG_H_
#define DFQ_DIAG_H_

#include "dfq_hip.h"

#ifdef __cplusplus
extern "C" {
#endif
/* The library is built with hidden visibility: only these entry points are
 * exported (two builds in one process -- the product and the diagnostics
 * library -- then never bind to each other's internals). */
#pragma GCC visibility push(default)

/* ---- measurement --------------------------------------------------------
 * Same-mix streaming probe (no arithmetic): y = x, codes = bits of x, esum = x,
 * n elements (multiple of 4); blocks < 0 selects a 4-deep variant with -blocks
 * blocks (n multiple of 16).  Used by bench.py as the achievable ceiling for
 * the sweep's traffic mix; not part of the reference interface. */
int dfq_probe_stream(const float* x, float* y, void* codes, float* esum, int64_t n, int32_t blocks,
                     void* stream);
/* Per-task timeline of sweep variant 13 (DFQ_SWEEP_VARIANT=13): 4 uint64 per
 * main-list task {start, data landed, done (s_memrealtime, 100 MHz), xcc<<32|hw_id};
 * buf NULL / cap 0 disables. */
int dfq_debug_timeline(void* buf, int64_t cap);
// Sweep variant 13 ablations (1 no row reduce, 2 stores without the quantize
// arithmetic, 4 no quantize loop, 8 no input loads, 16 the launch alone, 32 task and
// tensor records without compute): attribution runs only, the outputs are wrong
// while any bit is set.
int dfq_debug_ablate(uint32_t flags);
/* The sweep's memory pattern without arithmetic: 2048-element wave tasks through
 * LDS-DMA, non-temporal dq / codes / E stores (copy_only: dq only).  n % 2048 == 0. */
int dfq_probe_lds(const float* x, float* y, void* codes, float* esum, int64_t n, int32_t copy_only,
                  int32_t blocks, void* stream);

/* ---- structure checks ------------------------------------------------------
 * The CLE plan structure dfq_cle_plan_create builds for these relations and targets
 * (host code only: no device memory is touched, addresses may be stand-ins) checked
 * for every index its kernels derive from it -- task tables, range words, rollback
 * saves, metric chunks / units, the lagged placement windows and the stop rule's
 * offset (dfq_cle.hip).  info[8]: steps, nlaunch, lagged, stop_off, rescale tasks,
 * range tasks, units, chunks.  DFQ_ERR_INVALID + msg: the first violation.  Reads
 * the same diagnostics schedule switches as plan creation (DFQ_CLE_LAG, ...). */
int dfq_diag_cle_check_structure(const dfq_cle_rel* rels, int32_t n_rel, float* const* targets,
                                 const int64_t* target_n, int32_t n_targets, int32_t ref_threads, int64_t* info,
                                 char* msg, int32_t msg_cap);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif /* DFQ_DIAG_H_ */

/*
 * grace_hip.h — C ABI of the MI355X-native gradient-codec engine (libgrace_hip.so, gfx950).
 *
 * This is the drop-in boundary that replaces the reference's native bindings and the ATen
 * calls on its hot path (sands-lab/grace, grace_dl/dist):
 *   - qsgd_cuda.compress / decompress   grace_dl/dist/compressor/qsgd_cuda/qsgd.cpp:12-24
 *   - cnat_cuda.compress / decompress   grace_dl/dist/compressor/cnat_cuda/cnat.cpp:25-29
 *   - rdxtopk.topk                      grace_dl/dist/compressor/radixtopk_cuda/rdxtopk.cpp:11-18
 *   - the torch ops inside Compressor.compress/decompress and Memory.compensate/update
 *     (the grace_dl/dist/compressor and grace_dl/dist/memory modules).
 *
 * Rules for every entry point:
 *   - plain pointers to DEVICE memory allocated by the caller, element counts, and a hipStream_t
 *     passed as `void* stream` (NULL = legacy default stream);
 *   - all work is stream-ordered: nothing allocates, frees or synchronises, so the calls can be
 *     captured into a hipGraph;
 *   - scratch comes from a caller-provided workspace whose size is given by the matching
 *     *_workspace_bytes() query; zero it once when it is allocated.  Every entry point leaves the
 *     counters it uses zeroed, at offsets that do not depend on the call's sizes, so one workspace
 *     (at least as large as each call's query) serves calls of any shape on its stream;
 *   - return value is a grace_status_t (0 = launched OK, negative = error; see grace_last_error()).
 *   - f32 arithmetic follows the reference's torch ops exactly (no FMA contraction) unless a
 *     function's comment states a tolerance.
 */
#ifndef GRACE_HIP_H
#define GRACE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int grace_status_t;
#define GRACE_OK 0
#define GRACE_ERR_ARG (-1)
#define GRACE_ERR_HIP (-2)
#define GRACE_ERR_WORKSPACE (-3)

/* ---------------------------------------------------------------------------------- library */
int grace_version(void);
const char* grace_last_error(void);
/* Diagnostics (tests only; synchronises the stream): the device-side status word of the last
 * top-k launch on `workspace` (0 = sampled fast path, 1 = exact fallback, 2 = the parallel
 * exact fallback aborted after a wait ran out: see grace_topk_status_word). */
grace_status_t grace_read_status(const void* workspace, int32_t* status_host, void* stream);

/* The streaming skeleton of the headline main pass (bench.py's HBM ceiling): topk_main with the
 * same chunking, loads, stores and grid, but no classification -- r' = r + g and (sparse == 0)
 * out = 0 written in place; sparse != 0 is the recycled-output layout (out untouched).  Its rate
 * is the ceiling of the real pass's exact memory layout. */
size_t grace_topk_stream_probe_workspace_bytes(int64_t n);
/* Plain device allocations for the buffer-pair placement probe's spacers (grace_amd/ops.py
 * pick_pair): hipMalloc / hipFree, so the caller's allocator cache holds none of it.  A failed
 * allocation returns GRACE_ERR_HIP with *ptr = NULL. */
grace_status_t grace_spacer_alloc(size_t bytes, void** ptr);
grace_status_t grace_spacer_free(void* ptr);
grace_status_t grace_topk_stream_probe(const float* g, float* r, float* out, int64_t n, int32_t sparse, void* ws,
                                       size_t ws_bytes, void* stream);

/* Atomically read and clear a pinned host status word that kernels set bits in (system-scope
 * fetch_or): returns the bits set since the last take.  Host only, never blocks. */
int32_t grace_status_take(int32_t* host_word);

/* Top-k exact-fallback health.  grace_topk_status_word registers a pinned,
 * device-accessible host word (NULL unregisters) that every later top-k launch of this process
 * reports to: bit 2 = a wait of the parallel exact fallback ran out, so that launch's payload /
 * residual / output are NOT valid (the fallback aborted in every workgroup; its waits are only on
 * slices that running workgroups claimed, so this is never expected).  The device status word of
 * grace_read_status then reads 2.  grace_topk_fallback_spin_limit sets the bound of each of those
 * waits in microseconds of device wall time (default 2,000,000 = 2 s: only a true hang trips it;
 * limit < 0: unchanged) and returns the previous bound; tests set 0 to force a run-out.  The
 * launch's own results are already invalid when the word reports it: a caller that needs the
 * failing step itself to raise checks the word after that step's event (TopKCompressor
 * check_sync=True); otherwise the next top-k call raises. */
grace_status_t grace_topk_status_word(int32_t* host_word);
int64_t grace_topk_fallback_spin_limit(int64_t limit);

/* Event timer on the kernel's own stream, used by bench.py to time the dominant kernel of a
 * fused step: when enabled, that kernel's launch is bracketed by hipEventRecord. */
grace_status_t grace_timer_enable(int enable);
grace_status_t grace_timer_collect(float* total_ms, int32_t* launches);

/* Cross-bucket overlap: an event that completes with the MAIN pass of a top-k step, so
 * that the next bucket's step on another stream can start its bracket while this bucket's
 * finalize runs.  grace_topk_arm_main_event arms `event` for the next top-k step launched from
 * the calling thread (one-shot; the event rides on the main pass's dispatch packet, no marker).
 * Events come from grace_event_create (no system fence, no timing). */
grace_status_t grace_event_create(void** event);
grace_status_t grace_event_destroy(void* event);
grace_status_t grace_topk_arm_main_event(void* event);
grace_status_t grace_stream_wait_event(void* stream, void* event);

/* ------------------------------------------------------------------------ elementwise memory */
/* t = beta * r + gamma * g  (ResidualMemory.compensate, grace_dl/dist/memory/residual.py:10-14;
 * EFSignSGDMemory.compensate with beta = 1, gamma = lr, memory/efsignsgd.py:11-13) */
grace_status_t grace_axpby(const float* r, const float* g, float beta, float gamma, float* t,
                           int64_t n, void* stream);
/* r = t - d  (Memory.update residual, residual.py:18-20) */
grace_status_t grace_sub(const float* t, const float* d, float* r, int64_t n, void* stream);
/* out = x / divisor  (Communicator average: allgather.py:45, allreduce.py:12) */
grace_status_t grace_div_scalar(const float* x, float divisor, float* out, int64_t n, void* stream);
grace_status_t grace_fill(float* x, float value, int64_t n, void* stream);
/* HBM ceiling probe for bench.py (no reference counterpart): r = r + g, o = 0 with non-temporal 16-B
   loads / stores (the top-k step's 2-read / 2-write dense traffic, none of its arithmetic).
   variant 0-2: chunks of 8192 / 12288 / 16384 elements per workgroup; 3-5: grid-stride over
   1024 / 2048 / 4096 workgroups.  variant 6-9: the encoders' mix, read g and write one byte per
   element to o (r unused): chunks of 8192 / 16384 elements, grid-stride over 2048 / 4096 workgroups.
   grace_hbm_probe_elems: the elements a launch covers (-1: bad). */
int64_t grace_hbm_probe_elems(int64_t n, int32_t variant);
grace_status_t grace_hbm_probe(float* r, const float* g, float* o, int64_t n, int32_t variant, void* stream);
/* Compressor.aggregate = Python sum() in rank order (grace_dl/dist/__init__.py:32-34):
 * first != 0: acc = 0.0f + x (so -0 -> +0), else acc = acc + x. */
grace_status_t grace_accumulate(float* acc, const float* x, int64_t n, int32_t first, void* stream);

/* --------------------------------------------------------------------------------- sign family */
/* signSGD codeword u8 = (x >= 0)  (grace_dl/dist/compressor/signsgd.py:15-16) */
grace_status_t grace_sign_encode(const float* x, uint8_t* codes, int64_t n, void* stream);
/* f32 = u8 * 2 - 1 (signsgd.py:21); optional scale (EF-signSGD: mean * (2s-1), efsignsgd.py:26-27):
 * scale_dev may be NULL (= 1) */
grace_status_t grace_sign_decode(const uint8_t* codes, const float* scale_dev, float* out, int64_t n,
                                 void* stream);
/* Majority vote over W rank-major codeword rows (signsgd.py:25-30 applied to W decodes):
 * out = (sum_w (2 c_w - 1) >= 0) ? +1 : -1, summed in rank order in f32. */
grace_status_t grace_sign_majority(const uint8_t* codes_wn, int32_t world, float* out, int64_t n,
                                   void* stream);
/* Signum: m = coef_g * g + coef_m * m_prev (in place; m = g on the first step), codes = (m >= 0)
 * (signum.py:19-23).  The caller passes coef_g = f32(1.0 - momentum) computed in double and
 * coef_m = f32(momentum), i.e. the two Python scalars as torch rounds them. */
grace_status_t grace_signum_encode(const float* g, float* momentum, int32_t has_prev, float coef_g,
                                   float coef_m, uint8_t* codes, int64_t n, void* stream);
/* Fused signSGD step at world 1: codes = (x>=0), out = 2 c - 1 (aggregate of a single decode). */
/* codes may be NULL (the world-1 step needs only the decoded output) */
grace_status_t grace_sign_step_w1(const float* x, uint8_t* codes, float* out, int64_t n, void* stream);

/* ------------------------------------------------------------------------------- reductions */
size_t grace_reduce_workspace_bytes(int64_t n);
/* mean(|x|) -> f32 on device (efsignsgd.py:18) */
grace_status_t grace_abs_mean(const float* x, int64_t n, float* out_dev, void* ws, void* stream);
/* one-bit statistics: mask0 = (x < 0) as u8, mean0 = mean(x[x<0]), mean1 = mean(x[~(x<0)])
 * (onebit.py:13-23); means written to out_dev[0..1] */
grace_status_t grace_onebit_encode(const float* x, int64_t n, uint8_t* mask0, float* means_dev,
                                   void* ws, void* stream);
/* out = mask0 * mean0 + notmask * mean1; quirk != 0 reproduces the dist flavour's uint8 `~`
 * (onebit.py:29: notmask = 255 - mask0) */
grace_status_t grace_onebit_decode(const uint8_t* mask0, const float* mean0_dev, const float* mean1_dev,
                                   int32_t quirk, float* out, int64_t n, void* stream);

/* --------------------------------------------------------------------------- top-k sparsifier */
/* Top-k of |t| with the deterministic tie rule (larger |t| first, NaN largest, lower index first
 * among equal |t|); same set as torch.topk(sorted=False) (topk.py:36) modulo ties at the k-th
 * value.  Payload layout = reference's [values f32[k], indices int32[k]] (topk.py:41-42). */
size_t grace_topk_workspace_bytes(int64_t n, int64_t k);
/* The world > 1 residual step with the new residual written to a SECOND buffer (ResidualMemory's
 * update, residual.py:16-20, allocates a new tensor too): reads g and r_in, writes r_out and the
 * payload; r_out = t - decompress(compress(t)) exactly as grace_topk_residual_step leaves the
 * residual in place, but the main pass zeroes its provisional picks at once and the finalize fixes
 * up only the candidates it decides otherwise (t stays recoverable from g and r_in), instead of
 * zeroing every selected position afterwards.  has_residual = 0: t = g (r_in unused).  carry as
 * grace_topk_residual_step_carry (kept with the residual it describes: r_out after this step). */
grace_status_t grace_topk_residual_step_swap(const float* g, const float* r_in, int32_t has_residual, float beta,
                                             float gamma, int64_t n, int64_t k, float* vals, int32_t* idx,
                                             float* r_out, float* carry, int64_t carry_len, int32_t carry_valid,
                                             void* ws, size_t ws_bytes, void* stream);
/* TopKCompressor.compress on its own: x is only read. */
grace_status_t grace_topk_compress(const float* x, int64_t n, int64_t k, float* vals, int32_t* idx,
                                   void* ws, size_t ws_bytes, void* stream);
/* Fused world-1 Communicator.step for TopK + NoneMemory (grace_dl/dist/__init__.py:47-51,
 * memory/none.py, allgather.py:40-45): the payload of grace_topk_compress and, in the same
 * streaming pass, out = (0 + zeros(n).scatter_(idx, vals)) / 1.  x is only read.  prev_idx
 * (may be NULL): recycled output, as grace_topk_residual_step_carry. */
grace_status_t grace_topk_step_dense(const float* x, int64_t n, int64_t k, float* vals, int32_t* idx,
                                     float* out, const int32_t* prev_idx, int64_t prev_count, void* ws,
                                     size_t ws_bytes, void* stream);
/* Fused Communicator.step for TopK + ResidualMemory (grace_dl/dist/__init__.py:47-51):
 *   t = beta*r + gamma*g (t = g when has_residual == 0), payload = topk(t), r <- t - decode(payload)
 *   out (may be NULL): the world-1 Allgather result, zeros with t scattered at the payload.
 * `residual` is updated in place (it may hold garbage when has_residual == 0). */
grace_status_t grace_topk_residual_step(const float* g, float* residual, int32_t has_residual,
                                        float beta, float gamma, int64_t n, int64_t k, float* vals,
                                        int32_t* idx, float* out, void* ws, size_t ws_bytes,
                                        void* stream);
/* grace_topk_residual_step plus a residual-sample carry (same results, bit for bit): `carry`
 * (f32[carry_len >= grace_topk_carry_size(n, k)], owned by the caller next to the residual) receives t at the
 * sampled bracket's positions and the step's selection threshold; on the next step of the SAME
 * residual, with carry_valid != 0, the bracket derives r' at those positions from it instead of
 * reading r (half its random DRAM reads; the same sample bit for bit).  A stale carry (the residual
 * changed in between) only misplaces the sampled bracket, whose exact fallback keeps the result
 * exact.  carry_size 0: no carry for this (n, k); carry NULL: the plain step.
 * Recycled output (prev_idx != NULL, out != NULL): `out` must hold exactly the result of an earlier
 * step of this call whose payload indices are prev_idx[0 .. prev_count) -- zero everywhere else,
 * unmodified since.  The step then zeroes those positions and writes only the elements it selects
 * instead of all n (same result, bit for bit; 4 B per element less traffic).  NULL: dense write. */
int64_t grace_topk_carry_size(int64_t n, int64_t k);
grace_status_t grace_topk_residual_step_carry(const float* g, float* residual, int32_t has_residual,
                                              float beta, float gamma, int64_t n, int64_t k, float* vals,
                                              int32_t* idx, float* out, float* carry, int64_t carry_len,
                                              int32_t carry_valid, const int32_t* prev_idx, int64_t prev_count,
                                              void* ws, size_t ws_bytes, void* stream);
/* zeros(n).scatter_(idx, vals)  (topk.py:45-49; threshold.py:25-26; randomk.py:39-40). */
grace_status_t grace_sparse_decode(const float* vals, const int32_t* idx, int64_t count, float* out,
                                   int64_t n, void* stream);
grace_status_t grace_sparse_decode_i64(const float* vals, const int64_t* idx, int64_t count,
                                       float* out, int64_t n, void* stream);
/* Decode + aggregate of W gathered sparse payloads, exactly ((0 + d_0) + d_1 + ...) / divisor in
 * rank order (allgather.py:40-45).  vals/idx are rank-major [world][stride]; counts_host[w] is
 * rank w's payload length.  tags is an int32[n] scratch array (no initialisation needed). */
/* world > 1 decode via chunk-grouped payloads (grace_amd/csrc/payload.hip): each rank groups its
 * own payload by 8192-element output chunk before the exchange (grace_sort_payload: counting sort
 * by chunk, n <= 2^28; ws = grace_sort_payload_workspace_bytes; ends_out[ceil(n / 8192)] receives
 * the end offset of every chunk's entries and is sent with the payload), then
 * grace_sparse_aggregate_sorted writes out = (((0 + d_0) + d_1) + ...) / divisor densely in one
 * pass over the output (no zero-fill, no per-rank scatter).  The grouped payload carries each
 * entry's offset inside its 8192-element chunk (u16, off_out) instead of its index: 6 B per entry
 * on the wire.  vals and ends of rank w start at w * stride 4-B words, its offsets at 2 w stride u16.
 * Indices must be unique within each payload. */
size_t grace_sort_payload_workspace_bytes(int64_t k, int64_t n);
grace_status_t grace_sort_payload(const float* vals, const int32_t* idx, int64_t k, int64_t n, float* vals_out,
                                  uint16_t* off_out, uint32_t* ends_out, void* ws, size_t ws_bytes, void* stream);
grace_status_t grace_sparse_aggregate_sorted(const float* vals, const uint16_t* off, const uint32_t* ends,
                                             int64_t stride, int32_t world, float divisor, float* out, int64_t n,
                                             void* stream);
/* as grace_sparse_aggregate with `out` already zero-filled by the caller (lets the fill overlap
 * the payload exchange); 1 <= world <= 64 */
grace_status_t grace_sparse_aggregate_into(const float* vals, const int32_t* idx, int64_t stride,
                                           const int64_t* counts_host, int32_t world, float divisor,
                                           float* out, int32_t* tags, int64_t n, void* stream);
grace_status_t grace_sparse_aggregate(const float* vals, const int32_t* idx, int64_t stride,
                                      const int64_t* counts_host, int32_t world, float divisor,
                                      float* out, int32_t* tags, int64_t n, void* stream);

/* ------------------------------------------------------------------------------ quantisers */
/* Segmented buckets: x is one flat f32 buffer holding nseg tensors; seg_off[nseg + 1] (device)
 * gives their element offsets.  A single tensor is nseg = 1, seg_off = {0, n}.
 * Randomness: u (uniform [0,1) per element, the reference's torch stream) may be injected; when
 * NULL a counter-based device generator keyed by `seed` is used. */

/* QSGD (grace_dl/dist/compressor/qsgd.py:12-39; variant 1 = QSGDCompressor_CUDA semantics of
 * qsgd_cuda.cu:320-388).  bkt_off[nseg + 1] (device) = per-segment bucket offsets, bucket =
 * ceil(n_s / bucket_size) per segment; norms_out[nbuckets] f32; codes int8 (q < 128) or fp16.
 * norms_in (optional) injects the bucket norms (parity of codewords). */
/* World-1 Allgather(QSGD, NoneMemory).step with bucket_size 128 in one pass: out = 0 + (norm / q) *
 * code for the codes grace_qsgd_compress would produce (same seed / u), never stored; nseg <=
 * grace_qsgd_seg_max(). */
grace_status_t grace_qsgd_step_w1(const float* x, const int64_t* seg_off, const int64_t* bkt_off, int32_t nseg,
                                  int64_t nbuckets, int32_t quantum_num, int32_t variant, const float* u,
                                  uint64_t seed, float* out, void* stream);
int32_t grace_qsgd_seg_max(void);
grace_status_t grace_qsgd_compress(const float* x, const int64_t* seg_off, const int64_t* bkt_off,
                                   int32_t nseg, int64_t nbuckets, int32_t quantum_num, int32_t bucket_size,
                                   int32_t variant, const float* u, uint64_t seed, const float* norms_in,
                                   float* norms_out, void* codes, void* stream);
/* The same on a shard of a larger bucket (grace_amd/dist/sharded_quant.py): x[0] is the bucket's
 * element xoff (0 <= xoff < 2^31) and the shard starts on a bucket boundary of its first segment;
 * the device generator draws by the bucket's element index, so the codes equal the whole-bucket
 * call's codes for the shard's elements. */
grace_status_t grace_qsgd_compress_at(const float* x, int64_t xoff, const int64_t* seg_off, const int64_t* bkt_off,
                                      int32_t nseg, int64_t nbuckets, int32_t quantum_num, int32_t bucket_size,
                                      int32_t variant, const float* u, uint64_t seed, const float* norms_in,
                                      float* norms_out, void* codes, void* stream);
/* (norm / q) * code (qsgd.py:44-49).  world > 1 with rank-major payload strides: decode +
 * aggregate in rank order, aggregate != 0 adds the Python-sum 0 (allgather.py:40-45); divisor
 * applies the average. */
grace_status_t grace_qsgd_decompress(const void* codes, const float* norms, int64_t code_stride,
                                     int64_t norm_stride, int32_t world, const int64_t* seg_off,
                                     const int64_t* bkt_off, int32_t nseg, int64_t n, int32_t quantum_num,
                                     int32_t bucket_size, int32_t variant, int32_t aggregate, float divisor,
                                     float* out, void* stream);
/* Sharded QSGD (grace_amd/dist/sharded_quant.py, bucket_size 128): the whole bucket decoded straight
 * from the W gathered per-rank records (no copy into flat code / norm buffers).  Rank w holds the
 * buckets [w U, (w + 1) U) (U = units_per_rank) and the elements from rank_lo[w] (device int64[W]);
 * its record starts at records + w * rec_bytes with the codes of its elements from byte 0 and the
 * f32 norms of its buckets from byte norm_off_bytes (both 16-B multiples).  Same arithmetic as
 * grace_qsgd_decompress at world 1. */
grace_status_t grace_qsgd_decompress_records(const void* records, int64_t rec_bytes, int64_t norm_off_bytes,
                                             int32_t world, int64_t units_per_rank, const int64_t* rank_lo,
                                             const int64_t* seg_off, const int64_t* bkt_off, int32_t nseg, int64_t n,
                                             int32_t quantum_num, int32_t variant, float* out, void* stream);
/* QSGD, Horovod flavour (grace_dl/torch/compressor/qsgd.py:12-31): ONE norm over the whole tensor
 * (tensor.norm(); no buckets), same codeword rule.  norm_out[1] f32 (f64 accumulation), norm_in
 * (optional) injects it; ws = grace_qsgd_global_workspace_bytes().  Decode with
 * grace_qsgd_decompress, one segment of one bucket of n elements (qsgd.py:33-38: norm / q * code). */
size_t grace_qsgd_global_workspace_bytes(void);
grace_status_t grace_qsgd_global_compress(const float* x, int64_t n, int32_t quantum_num, const float* u,
                                          uint64_t seed, const float* norm_in, float* norm_out, void* codes,
                                          void* ws, void* stream);
/* TernGrad (terngrad.py:7-30).  unit_off[nseg + 1] (device) = per-segment offsets of
 * grace_terngrad_unit()-element work units; ws = grace_terngrad_workspace_bytes(nunits).
 * clip_in[nseg] (optional) injects the clamp bound c = f32(2.5 * std). */
int32_t grace_terngrad_unit(void);
size_t grace_terngrad_workspace_bytes(int64_t nunits);
grace_status_t grace_terngrad_compress(const float* x, const int64_t* seg_off, const int64_t* unit_off,
                                       int32_t nseg, int64_t nunits, const float* clip_in, const float* u,
                                       uint64_t seed, int8_t* codes, float* scalars, void* ws,
                                       void* stream);
/* World-1 Allgather(TernGrad, NoneMemory).step: the statistics pass, then ONE pass writing
 * out = 0 + code * scalar for the codes grace_terngrad_compress would produce (same seed / u / clip)
 * without storing them; scalars[nseg] are still written.  16-B aligned x and out. */
grace_status_t grace_terngrad_step_w1(const float* x, const int64_t* seg_off, const int64_t* unit_off, int32_t nseg,
                                     int64_t nunits, const float* clip_in, const float* u, uint64_t seed,
                                     float* scalars, void* ws, float* out, void* stream);
/* Sharded TernGrad (grace_amd/dist/sharded_terngrad.py).  One bucket's work units are
 * split over the ranks in contiguous blocks; a rank runs the GLOBAL units [unit0, unit0 +
 * nunits_local) of the bucket's tables, whose elements start at global element xoff (x, u and codes
 * point there, 16-B aligned).  ws = the GLOBAL slot array (grace_terngrad_workspace_bytes(nunits),
 * grace_terngrad_slot_bytes() per unit): shard_stats writes this rank's units' slots; after the
 * caller has all-gathered every rank's slots into it, shard_encode writes this rank's codes with
 * every segment's scale reduced exactly as the single-GPU encoder (bit-identical codes when every
 * unit starts on a multiple of 4 elements; a unit at another offset sums its f64 partials in another
 * quad phase, so the clip and scalar may differ by an ulp, rarely), and
 * grace_terngrad_scalars derives every segment's scalar the same way (nothing but the slots
 * travels before the codes). */
/* Sharded TernGrad's replicated decode straight from the W gathered records: rank w's codes of the
 * elements [rank_lo[w], rank_lo[w + 1]) (device int64[W + 1], W <= 64) at records + w * rec_bytes,
 * int8 (packed = 0) or code + 1 in the 2-bit planar layout of grace_tern_pack (packed = 1);
 * out = code * scalars[segment], as grace_terngrad_decompress at world 1.  16-B aligned records and
 * out, rec_bytes a 16-B multiple, nseg <= grace_qsgd_seg_max(). */
grace_status_t grace_terngrad_decompress_records(const void* records, int64_t rec_bytes, int32_t world,
                                                 const int64_t* rank_lo, int32_t packed, const float* scalars,
                                                 const int64_t* seg_off, int32_t nseg, int64_t n, float* out,
                                                 void* stream);
int32_t grace_terngrad_slot_bytes(void);
grace_status_t grace_terngrad_shard_stats(const float* x, int64_t xoff, const int64_t* seg_off,
                                          const int64_t* unit_off, int32_t nseg, int64_t unit0, int64_t nunits_local,
                                          void* ws, void* stream);
grace_status_t grace_terngrad_shard_encode(const float* x, int64_t xoff, const int64_t* seg_off,
                                           const int64_t* unit_off, int32_t nseg, int64_t unit0,
                                           int64_t nunits_local, const float* clip_in, const float* u, uint64_t seed,
                                           int8_t* codes, const void* ws, void* stream);
grace_status_t grace_terngrad_scalars(const int64_t* seg_off, const int64_t* unit_off, int32_t nseg,
                                      const float* clip_in, const void* ws, float* scalars, void* stream);
grace_status_t grace_terngrad_decompress(const int8_t* codes, const float* scalars, int64_t code_stride,
                                         int64_t scal_stride, int32_t world, const int64_t* seg_off,
                                         int32_t nseg, int64_t n, int32_t aggregate, float divisor, float* out,
                                         void* stream);
/* natural compression: cupy flavour (natural.py:12-29; rand_int = randint(0, 2^23-1) stream) and
 * cnat_cuda flavour (cnat_cuda.cu:68-123; rand = uniform stream, or deterministic threshold 0.5). */
grace_status_t grace_natural_compress(const float* x, int64_t n, const int32_t* rand_int, uint64_t seed,
                                      uint8_t* codes, void* stream);
grace_status_t grace_cnat_compress(const float* x, int64_t n, const float* rand, int32_t deterministic,
                                   uint64_t seed, uint8_t* codes, void* stream);
/* the same on a shard of a larger bucket: x[0] is its element xoff (a multiple of 4) for the device
 * generator (grace_amd/dist/sharded_quant.py) */
grace_status_t grace_natural_compress_at(const float* x, int64_t xoff, int64_t n, const int32_t* rand_int,
                                         uint64_t seed, uint8_t* codes, void* stream);
grace_status_t grace_cnat_compress_at(const float* x, int64_t xoff, int64_t n, const float* rand,
                                      int32_t deterministic, uint64_t seed, uint8_t* codes, void* stream);
/* flavour 0 = natural.py:35-39 decode, 1 = cnat_cuda.cu:125-134 decode */
grace_status_t grace_natural_decompress(const uint8_t* codes, int64_t stride, int32_t world, int64_t n,
                                        int32_t flavour, int32_t aggregate, float divisor, float* out,
                                        void* stream);
/* fp16 (fp16.py): round-to-nearest-even cast and back */
grace_status_t grace_fp16_compress(const float* x, void* half_out, int64_t n, void* stream);
grace_status_t grace_fp16_decompress(const void* half_in, float* out, int64_t n, void* stream);
/* World-1 Allgather(compressor, NoneMemory).step of an element-wise codec in one pass:
 * out = 0 + decompress(compress(x)); mode 0 natural (device generator keyed by seed, the
 * grace_natural_compress stream), 1 cnat (grace_cnat_compress's device stream), 2 cnat
 * deterministic, 3 fp16.  The codes are the separate compress kernels' bit for bit. */
grace_status_t grace_cast_step_w1(const float* x, int64_t n, int32_t mode, uint64_t seed, float* out,
                                  void* stream);
/* Allgather step's decode of W rank-major f16 payloads (rank r at half_in + r * stride):
 * out = ((0 + d_0) + d_1 + ... + d_{W-1}) / divisor (no division when divisor == 1), one pass
 * (allgather.py:40-45 with fp16.py's decompress) */
grace_status_t grace_fp16_decompress_aggregate(const void* half_in, int64_t stride, int32_t world, int64_t n,
                                               float divisor, float* out, void* stream);

/* Per-tensor top-k + residual over many tensors in one launch sequence (csrc/topk.hip "Segmented"):
 * the reference's per-parameter DDP loop (examples/dist/CIFAR10-dawndist/core.py:203-206, one
 * TopKCompressor(ratio) + ResidualMemory step per tensor, k_i = max(1, int(n_i * ratio)),
 * grace_dl/dist/compressor/topk.py:34).  The tensors are segments of one flat buffer; three launches
 * stream every element once: small segments (n <= grace_topk_segmented_small_max()) are selected
 * exactly in one workgroup each, large ones get a sampled bracket, one main pass over their chunks
 * and one finalize workgroup each (the single-bucket engine per segment).  Device tables:
 * seg_off[nseg + 1] (elements), k_off[nseg + 1] (payload), large[n_large] / small[n_small] (segment
 * ids), chk_off[n_large + 1] (main-pass chunks of grace_topk_segmented_chunk(has_residual,
 * out != NULL) elements per large segment), chunk_li[nchunks] (large slot of each chunk),
 * ws_off[n_large] (byte offsets of each large segment's grace_topk_segmented_seg_ws_bytes(n, k)
 * workspace, 256-B aligned, zeroed once), fin_off[n_large + 1] / fin_li[nfin] (the finalize
 * workgroups: grace_topk_segmented_fin_blocks(n, k) per large segment).  Payload (vals f32, idx i32 GLOBAL indices)[k_off[nseg]];
 * out (dense world-1 result, may alias g) or NULL (world > 1: residual and payload only).
 * carry (may be NULL; has_residual only): f32, grace_topk_segmented_carry_len(n) words per large
 * segment at carry_off[n_large] -- the segment's t at its sample positions and its selection
 * threshold, written by the step; carry_valid: they are the previous step's for this residual
 * (the next prep then reads g alone at the sample positions). */
int32_t grace_topk_segmented_small_max(void);
int64_t grace_topk_segmented_chunk(int32_t has_residual, int32_t dense_out);
int64_t grace_topk_segmented_seg_ws_bytes(int64_t n, int64_t k);
int32_t grace_topk_segmented_fin_blocks(int64_t n, int64_t k);
/* The workspace a segment table needs (host arrays sizes[count], ks[count]: the LARGE segments,
 * those listed in `large`): the sum of their 256-B aligned grace_topk_segmented_seg_ws_bytes.  Pass
 * it as ws_need: the step refuses ws_bytes < ws_need (the per-segment offsets ws_off are
 * device tables the host call cannot read). */
int64_t grace_topk_segmented_workspace_bytes(const int64_t* sizes, const int64_t* ks, int32_t count);
grace_status_t grace_topk_segmented_step(const float* g, float* residual, int32_t has_residual, float beta,
                                         float gamma, const int64_t* seg_off, const int64_t* k_off,
                                         const int32_t* large, int32_t n_large, const int32_t* small,
                                         int32_t n_small, const int64_t* chk_off, const int32_t* chunk_li,
                                         int64_t nchunks, const int64_t* ws_off, const int64_t* fin_off,
                                         const int32_t* fin_li, int64_t nfin, int64_t n_total, float* vals,
                                         int32_t* idx, float* out, float* carry, const int64_t* carry_off,
                                         int32_t carry_valid, void* ws, size_t ws_bytes, int64_t ws_need,
                                         void* stream);
int64_t grace_topk_segmented_carry_len(int64_t n);

/* ---------------------------------------------------------------------- random-k / threshold */
/* Random-k indices (randomk.py:11: randint(numel, [k]), WITH replacement) from a counter-based
 * device generator keyed by the reference's seed sum(bytes(name)) + step: identical on every
 * rank.  (Bit-parity with torch's CPU generator: draw on the host and pass the indices.) */
grace_status_t grace_randomk_indices(uint64_t seed, int64_t numel, int64_t k, int64_t* idx, void* stream);
/* Random-k, Horovod flavour (grace_dl/torch/compressor/randomk.py:10: randperm(numel)[:k], WITHOUT
 * replacement): idx[j] = pi(j), pi a keyed pseudorandom permutation of [0, numel) (Feistel network
 * + cycle walking), so the k indices are distinct; identical on every rank for the same seed. */
grace_status_t grace_randomk_perm_indices(uint64_t seed, int64_t numel, int64_t k, int64_t* idx, void* stream);
/* dst[j] = (int64)src[j]: int64 index payloads of the Horovod-flavour top-k
 * (grace_dl/torch/compressor/topk.py:11 keeps torch.topk's int64 indices) */
grace_status_t grace_widen_i32(const int32_t* src, int64_t n, int64_t* dst, void* stream);
/* vals[j] = x[idx[j]]  (randomk.py:12 tensor[indices]) */
grace_status_t grace_gather(const float* x, const int64_t* idx, int64_t k, float* vals, void* stream);
/* World-1 Allgather(RandomK, ResidualMemory).step (randomk.py:24-41, residual.py:10-20): with the
 * caller's idx[k] (grace_randomk_indices or torch's stream), t = beta r + gamma g (t = g when
 * has_residual == 0), vals = t[idx], residual <- t - decode(vals), out = (0 + decode(vals)) / 1. */
grace_status_t grace_randomk_step_w1(const float* g, float* residual, int32_t has_residual, float beta, float gamma,
                                     int64_t n, const int64_t* idx, int64_t k, float* vals, float* out,
                                     void* stream);
/* Sharded random-k + residual (grace_amd/dist/sharded_randomk.py): this rank holds the bucket's
 * elements [lo, lo + m) (g, residual and out point there); idx[k] are the bucket's GLOBAL indices,
 * the same on every rank.  residual <- t with this rank's drawn positions t - t; vals[j] = t at
 * idx[j] if this rank holds it, else +0 (the ranks' vals sum to the whole bucket's payload);
 * out (may be NULL): this rank's slice of the world-1 step's result, 0 + t at its drawn positions. */
grace_status_t grace_randomk_shard_step(const float* g, float* residual, int32_t has_residual, float beta, float gamma,
                                       int64_t lo, int64_t m, const int64_t* idx, int64_t k, float* vals, float* out,
                                       void* stream);
/* The world-1 step's result from the whole bucket's payload: out = zeros(n), out[idx[j]] = 0 + vals[j]
 * (randomk.py:39-40 decompress, allgather.py:44 sum from 0). */
grace_status_t grace_randomk_decode(const float* vals, const int64_t* idx, int64_t k, float* out, int64_t n,
                                    void* stream);
/* The same world-1 step without materialising the payload (only `out` is the step's result at
 * world 1): the indices are grouped by 8192-element chunk, then ONE streaming pass writes r' and
 * out (16 B per element, no random gathers / scatters); bit-identical out and r'.  n < 2^31 and
 * n <= 2^28; ws: grace_randomk_step_w1_dense_workspace_bytes, zeroed once at allocation.
 * grp (may be NULL): a caller-owned buffer of grace_randomk_group_bytes(n, k) that receives this
 * step's grouping of the indices.  prev_grp (may be NULL, needs grp): recycled output -- `out`
 * holds exactly the result of the earlier step whose grouping prev_grp is, unmodified since; its
 * non-zeros that are not drawn again are cleared and only the drawn positions are written. */
size_t grace_randomk_step_w1_dense_workspace_bytes(int64_t n, int64_t k);
size_t grace_randomk_group_bytes(int64_t n, int64_t k);
grace_status_t grace_randomk_step_w1_dense(const float* g, float* residual, int32_t has_residual, float beta,
                                           float gamma, int64_t n, const int64_t* idx, int64_t k, float* out,
                                           void* grp, const void* prev_grp, void* ws, size_t ws_bytes,
                                           void* stream);
/* Threshold (threshold.py:16-19): idx = where(|x| >= min(thr, max(x))) in ascending order.
 * count -> (host reads meta = ws[0..2]: bound bits, count, recount flag) -> [recount] -> write.
 * The caller synchronises once to size the variable-length payload. */
size_t grace_threshold_workspace_bytes(int64_t n);
grace_status_t grace_threshold_count(const float* x, int64_t n, float thr, void* ws, void* stream);
grace_status_t grace_threshold_recount(const float* x, int64_t n, float bound, void* ws, void* stream);
grace_status_t grace_threshold_write(const float* x, int64_t n, const void* ws, float* vals, int32_t* idx,
                                     void* stream);
/* count with the max(x) < thr recount decided on the device (ws[4..8] = final count): the count can be
 * exchanged between ranks before the host reads anything (one host read per variable-size step) */
grace_status_t grace_threshold_count_dev(const float* x, int64_t n, float thr, void* ws, void* stream);
/* r[idx[j]] -= vals[j] (ResidualMemory.update, residual.py:16-20, when r already holds t) */
/* World-1 Allgather(Threshold, ResidualMemory | NoneMemory).step without a payload
 * (threshold.py:12-27, residual.py:10-20, allgather.py:40-45): mode 0 no memory (t = g), 1 residual
 * memory's first step (t = g copied into residual), 2 t = beta r + gamma g (in place in residual);
 * out = (|t| >= min(thr, max t) ? 0 + t : 0), residual <- t - decode.  ws as grace_threshold_count. */
grace_status_t grace_threshold_step_w1(const float* g, float* residual, int32_t mode, float beta, float gamma,
                                       int64_t n, float thr, void* ws, float* out, void* stream);
grace_status_t grace_sparse_sub(const float* vals, const int32_t* idx, int64_t count, float* r, void* stream);
/* Capacity-bounded variable-size exchange (allgather.py:15-38 without the size round trip): each rank
 * writes one record of grace_exchange_record_words(cap) u32 words {count, cap, 0, 0 | vals f32[cap] |
 * idx i32[cap]} (entries past cap are dropped: overflow), the records are all-gathered as one
 * fixed-size buffer, and the aggregate reads the counts from the gathered headers on the device.
 * stat (device u32[2]) = {max count over ranks, overflow flag}: the same on every rank. */
size_t grace_exchange_record_words(int64_t cap);
grace_status_t grace_threshold_write_capped(const float* x, int64_t n, const void* ws, uint32_t* rec, int64_t cap,
                                            void* stream);
grace_status_t grace_sparse_aggregate_capped(const uint32_t* recs, int64_t stride, int64_t cap, int32_t world,
                                             float divisor, float* out, int32_t* tags, int64_t n, uint32_t* stat,
                                             void* stream);
/* r[idx] -= vals over the min(count, cap) entries of one record */
grace_status_t grace_sparse_sub_capped(const uint32_t* rec, int64_t cap, float* r, void* stream);
/* Horovod flavour (grace_dl/torch/compressor/threshold.py:17): where(|x| > thr), int64 indices.
 * bound = the smallest f32 above f32(thr) (|x| > thr <=> |x| >= bound), NaN for thr = +inf. */
grace_status_t grace_threshold_count_fixed(const float* x, int64_t n, float bound, void* ws, void* stream);
grace_status_t grace_threshold_write_i64(const float* x, int64_t n, const void* ws, float* vals, int64_t* idx,
                                         void* stream);

/* ---------------------------------------------------------------------------------- PowerSGD */
/* PowerSGD (powersgd.py:30-65) on M[n x m] row-major, rank r <= 16, f32 MFMA contractions.
 * P = M q and Q = M^T P share one workspace (grace_powersgd_workspace_bytes, zeroed once at
 * allocation, left zeroed by every call);  orthogonalize in place (Cholesky-QR, f64);
 * out = P Q^T and/or residual = M - P Q^T (memory/powersgd.py:32-37) in one pass. */
grace_status_t grace_powersgd_p(const float* M, int64_t n, int64_t m, const float* q, int32_t r, float* P,
                                void* ws, void* stream);
size_t grace_powersgd_workspace_bytes(int64_t n, int64_t m, int32_t r);
/* P = M q with q = standard normal draws keyed by `seed` (the grace_normal_fill stream of an [m x r]
 * tensor), drawn inside the contraction: no q buffer, no draw launch.  PowerSGD's fresh q
 * (powersgd.py:41-43) is orthogonalised before P = M q; since orthogonalize(M q R^-1) =
 * orthogonalize(M q) for the upper-triangular R of q's own QR, orthogonalize(P) is the same
 * either way, so the caller orthogonalises P only. */
grace_status_t grace_powersgd_p_draw(const float* M, int64_t n, int64_t m, uint64_t seed, int32_t r, float* P,
                                     void* ws, void* stream);
grace_status_t grace_powersgd_qt(const float* M, int64_t n, int64_t m, const float* P, int32_t r, float* Q,
                                 void* ws, void* stream);
grace_status_t grace_orthogonalize(float* A, int64_t n, int32_t r, void* stream);
/* q = orthogonalize(normal draws) in one launch (powersgd.py:41-43); same draws as grace_normal_fill */
grace_status_t grace_normal_orthogonal(float* A, int64_t n, int32_t r, uint64_t seed, void* stream);
grace_status_t grace_powersgd_outer(const float* P, const float* Q, int64_t n, int64_t m, int32_t r, float* out,
                                    const float* M, float* residual, void* stream);
/* World-size-1 rank-4 compress in one pass over M (replaces the P / orthogonalize / Qt sequence
 * of PowerSGDCompressor.compress, powersgd.py:30-56, when nothing is all-reduced in between):
 * P = orthogonalize(M q) and Q = M^T P, with q = `q` [m x 4] if non-null, else the standard normal
 * draws keyed by `seed` (the grace_normal_fill stream; as for grace_powersgd_p_draw, q itself need
 * not be orthogonalised).  Qraw = M^T (M q) is accumulated in f64 and solved by the R of P's QR.
 * Eligibility (grace_powersgd_w1_ok): r == 4, m % 4 == 0, m <= 16384, n <= 1 Mi rows; 16-B aligned
 * pointers.  The workspace (grace_powersgd_w1_workspace_bytes) is zeroed once at allocation and
 * left with its counters zeroed by every call.
 * The kernels hand data between workgroups with bounded waits on a grid of one workgroup per CU;
 * two such calls must not run concurrently (on two streams), or their grids could each hold CUs
 * the other one waits for.  `status_host` (optional, pinned host memory, never cleared by the
 * library) receives bit 1 when a wait ran out: that call's P and Q must not be used.  The caller
 * reads it after the stream has passed the call (grace_amd/ops.py checks it at every call and
 * orders calls issued on different streams). */
int32_t grace_powersgd_w1_ok(int64_t n, int64_t m, int32_t r);
size_t grace_powersgd_w1_workspace_bytes(int64_t n, int64_t m);
grace_status_t grace_powersgd_w1_compress(const float* M, int64_t n, int64_t m, const float* q, uint64_t seed,
                                          float* P, float* Q, void* ws, size_t ws_bytes, uint32_t* status_host,
                                          void* stream);
/* standard normal fill (q draws, powersgd.py:41 / memory/powersgd.py:27), device generator */
grace_status_t grace_normal_fill(float* x, int64_t n, uint64_t seed, void* stream);

/* ---- sharded top-k (BASELINE configs[4]) ------------------------------------
 * One bucket split into contiguous shards, one per rank; replaces the single-process
 * TopKCompressor.compress + ResidualMemory (grace_dl/dist/compressor/topk.py:32-42,
 * memory/residual.py:10-20) and the host-synced variable-size Allgather
 * (grace_dl/dist/communicator/allgather.py:15-38) for one bucket sharded over ranks.  Per step
 * (grace_amd/dist/sharded.py; csrc/shard.hip), no host synchronisation:
 *   grace_topk_residual_step(shard, k_loc = min(k, m)) into this rank's record
 *   [header (word 0 = m) | vals f32[cap] | local idx i32[cap], idx -1 = padding], cap = k
 *   -> ONE all_gather of the W records -> grace_shard_select.
 * grace_shard_select: the exact global top-k of the gathered entries (larger |t| first, lower
 * global index first, as the single-GPU engine): out[gi - out_base] = 0 + v for every selected
 * gi in [out_base, out_base + out_len) (out zero-filled by the caller); for this rank's record
 * entries pay_idx[j] = global index if selected, else -1, and the residual gets t back
 * (residual[idx] = v) where the local engine picked an entry the global cut rejects.
 * tab: device int64 [m_0 .. m_{W-1}, base_0 .. base_{W-1}] (the agreed partition).  status_host
 * (pinned, may be NULL): bit 1 = a record's shard length differs from tab, bit 2 = fewer valid
 * entries than k (both set with system-scope atomics; read them with grace_status_take).  sel_gi (may be
 * NULL): int32 [world * cap], every gathered entry's global index if selected, else -1 -- the
 * output's non-zero positions, which grace_shard_clear zeroes when the next step reuses `out`
 * (a recycled output, instead of a zero-fill of out_len elements). */
size_t grace_shard_record_words(int64_t cap);
size_t grace_shard_select_workspace_bytes(int32_t world, int64_t cap);
grace_status_t grace_shard_select(const int32_t* recs, int32_t world, int32_t rank, int64_t cap, const int64_t* tab,
                                  int64_t k, float* residual, float* out, int64_t out_base, int64_t out_len,
                                  int32_t* pay_idx, int32_t* sel_gi, void* ws, size_t ws_bytes, int32_t* status_host,
                                  void* stream);
grace_status_t grace_shard_clear(float* out, int64_t out_base, int64_t out_len, const int32_t* sel_gi, int64_t count,
                                 void* stream);

/* ---- DGC (grace_dl/dist/compressor/dgc.py:12-50, memory/dgc.py:15-39) -------------------------
 * compress: grace_dgc_sample (|t| at the sampled indices: sample_idx from the caller = torch's
 * CPU uniform_(0, numel).long() stream, or NULL = device generator) -> thr0, the k_s-th largest of the
 * sample (grace_dgc_sample_kth; or the k_s largest by grace_topk_compress) -> grace_dgc_threshold (sampled threshold, the 10-step adjustment
 * replayed on exact counts, ordered-compaction offsets; the selected count is at ws + 8, u32)
 * -> grace_dgc_write (values f32, indices int64, ascending).  The final threshold's bits are at
 * ws + 4 (u32); grace_dgc_mask_update reads them from the first 16 bytes of `meta`. */
size_t grace_dgc_workspace_bytes(int64_t n);
grace_status_t grace_dgc_sample(const float* t, int64_t n, const int64_t* sample_idx, uint64_t seed, int64_t ns,
                                float* sample_abs, void* stream);
grace_status_t grace_dgc_threshold(const float* t, int64_t n, const float* top_vals, int64_t ks, double ratio,
                                   void* ws, void* stream);
grace_status_t grace_dgc_write(const float* t, int64_t n, const void* ws, float* vals, int64_t* idx, void* stream);
/* Capacity-bounded exchange (no reference counterpart; replaces the size round trip of
   grace_dl/dist/communicator/allgather.py:15-38 for DGC): after grace_dgc_threshold, write this rank's
   record {count, cap, 0, 0 | vals f32[cap] | idx i32[cap]} (grace_exchange_record_words(cap) words),
   entries past cap dropped; aggregate the gathered records with grace_sparse_aggregate_capped. */
grace_status_t grace_dgc_write_capped(const float* t, int64_t n, const void* ws, uint32_t* rec, int64_t cap,
                                      void* stream);
/* DgcMemory.update (grace_dl/dist/memory/dgc.py:21-28) over the record's entries: r[i] *= 0, a[i] *= 0. */
grace_status_t grace_dgc_mask_update_capped(const uint32_t* rec, int64_t cap, float* residual, float* accum,
                                            void* stream);
/* memory: r = m r + g, a = a + r (has_state 0: r = a = g);  update: r *= keep, a *= keep with
 * keep = !(|t| >= thr) (t may alias a) */
grace_status_t grace_dgc_compensate(const float* g, float* residual, float* accum, int32_t has_state,
                                    float momentum, int64_t n, void* stream);
grace_status_t grace_dgc_mask_update(const float* t, float* residual, float* accum, int64_t n, const void* meta,
                                     void* stream);
/* grace_dgc_threshold without the payload bookkeeping: the sampled threshold and the 10-step
 * adjustment only (meta at ws). */
grace_status_t grace_dgc_select(const float* t, int64_t n, const float* top_vals, int64_t ks, double ratio, void* ws,
                                void* stream);
/* World-1 Allgather(DgcCompressor, DgcMemory).step after grace_dgc_select: DgcMemory.update
 * (r *= keep, a *= keep) and out = (0 + decompress(payload)) / 1 = (|t| >= thr ? 0 + t : 0) in one
 * pass; the payload and its host-read size are never materialised.  t may alias accum. */
grace_status_t grace_dgc_step_w1(const float* t, float* residual, float* accum, int64_t n, const void* ws, float* out,
                                 void* stream);
/* World-1 Allgather(DgcCompressor, DgcMemory(momentum, clipping off)).step from the OLD memory
 * state in one streaming pass (compressor/dgc.py:12-50, memory/dgc.py:15-39, allgather.py:40-45):
 * grace_dgc_sample_comp samples |t| of t = a + (m r + g) (t = g when has_state == 0) without
 * materialising t; with top_vals = the ks largest sampled magnitudes, grace_dgc_step_w1_fused
 * writes the new residual / accumulator (residual_out, accum_out: new buffers, the old state is
 * only read) and out = (0 + decompress) / 1.  It selects at the sampled threshold and checks the
 * reference's adjustment loop on the exact count; when that threshold does not stand, gated
 * launches redo the step with the full loop (same results as grace_dgc_compensate +
 * grace_dgc_select + grace_dgc_step_w1, bit for bit).  ws: grace_dgc_step_w1_fused_workspace_bytes,
 * zeroed once at allocation. */
grace_status_t grace_dgc_sample_comp(const float* g, const float* residual, const float* accum, int32_t has_state,
                                     float momentum, int64_t n, const int64_t* sample_idx, uint64_t seed, int64_t ns,
                                     float* sample_abs, void* stream);
/* out[0] = the ks-th largest of sample_abs[0..ns) (magnitudes: the sign bit is ignored), NaN when
 * any sample is NaN: torch.topk(samples, ks)[0].min() of dgc.py:20-21 without the full top-k, to
 * pass to grace_dgc_threshold / _select / _step_w1_fused as top_vals with ks = 1.
 * 1 <= ks <= ns < 2^32.  ws: grace_dgc_sample_kth_workspace_bytes, zeroed once at allocation (left
 * zeroed by every call). */
size_t grace_dgc_sample_kth_workspace_bytes(void);
grace_status_t grace_dgc_sample_kth(const float* sample_abs, int64_t ns, int64_t ks, void* ws, float* out,
                                    void* stream);
size_t grace_dgc_step_w1_fused_workspace_bytes(int64_t n);
grace_status_t grace_dgc_step_w1_fused(const float* g, const float* residual, const float* accum, int32_t has_state,
                                       float momentum, int64_t n, const float* top_vals, int64_t ks, double ratio,
                                       void* ws, float* residual_out, float* accum_out, float* out, void* stream);
/* gradient clipping (memory/dgc.py:16-19): s = sum(x*x) (f64 accumulate) into out_dev; after the
 * caller's all_reduce of s: out = clamp(x, -c, c), c = sqrt(s / world) */
size_t grace_sumsq_workspace_bytes(void);
grace_status_t grace_sumsq(const float* x, int64_t n, void* ws, float* out_dev, void* stream);
grace_status_t grace_clip_by_sumsq(const float* x, const float* sumsq_dev, float world, float* out, int64_t n,
                                   void* stream);

/* ---- packed wire formats ------------------------------------------------
 * 1-bit: sign codes u8 {0,1} <-> u32 words, bit i of the stream = code i (LSB first);
 * majority decode (signsgd.py:24-30) straight from W packed payloads (rank w at + w * stride).
 * 2-bit: grace_dl/tensorflow/compressor/packing.py:4-29 byte layout (planar quarters, pad values
 * range(0, 4 - n % 4)); grace_pack2_bytes(n) output bytes.  TernGrad codes travel as code + 1. */
grace_status_t grace_pack_bits(const uint8_t* codes, int64_t n, uint32_t* words, void* stream);
/* SignSGDCompressor.compress (signsgd.py:13-16) straight into the 1-bit layout: word i bit j =
 * (x[32 i + j] >= 0); the words grace_pack_bits would make from grace_sign_encode's codes. */
grace_status_t grace_sign_encode_bits(const float* x, int64_t n, uint32_t* words, void* stream);
grace_status_t grace_unpack_bits(const uint32_t* words, int64_t n, uint8_t* codes, void* stream);
grace_status_t grace_sign_majority_bits(const uint32_t* words, int64_t stride_words, int32_t world, int64_t n,
                                        float* out, void* stream);
int64_t grace_pack2_bytes(int64_t n);
grace_status_t grace_pack2(const uint8_t* values, int64_t n, uint8_t* packed, void* stream);
grace_status_t grace_unpack2(const uint8_t* packed, int64_t n, uint8_t* values, void* stream);
grace_status_t grace_tern_pack(const int8_t* codes, int64_t n, uint8_t* packed, void* stream);
grace_status_t grace_tern_unpack(const uint8_t* packed, int64_t n, int8_t* codes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GRACE_HIP_H */

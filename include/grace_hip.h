/*
 * grace_hip.h — C ABI of the MI355X-native gradient-codec engine (libgrace_hip.so, gfx950).
 *
 * This is the drop-in boundary that replaces the reference's native bindings and the ATen
 * calls on its hot path (sands-lab/grace, grace_dl/dist):
 *   - qsgd_cuda.compress / decompress   grace_dl/dist/compressor/qsgd_cuda/qsgd.cpp:12-24
 *   - cnat_cuda.compress / decompress   grace_dl/dist/compressor/cnat_cuda/cnat.cpp:25-29
 *   - rdxtopk.topk                      grace_dl/dist/compressor/radixtopk_cuda/rdxtopk.cpp:11-18
 *   - the torch ops inside Compressor.compress/decompress and Memory.compensate/update
 *     (grace_dl/dist/compressor/*.py, grace_dl/dist/memory/*.py).
 *
 * Rules for every entry point:
 *   - plain pointers to DEVICE memory allocated by the caller, element counts, and a hipStream_t
 *     passed as `void* stream` (NULL = legacy default stream);
 *   - all work is stream-ordered: nothing allocates, frees or synchronises, so the calls can be
 *     captured into a hipGraph;
 *   - scratch comes from a caller-provided workspace whose size is given by the matching
 *     *_workspace_bytes() query;
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
 * top-k launch on `workspace` (0 = sampled fast path, 1 = exact fallback). */
grace_status_t grace_read_status(const void* workspace, int32_t* status_host, void* stream);

/* Event timer on the kernel's own stream, used by bench.py to time the dominant kernel of a
 * fused step: when enabled, that kernel's launch is bracketed by hipEventRecord. */
grace_status_t grace_timer_enable(int enable);
grace_status_t grace_timer_collect(float* total_ms, int32_t* launches);

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
/* TopKCompressor.compress on its own: x is only read. */
grace_status_t grace_topk_compress(const float* x, int64_t n, int64_t k, float* vals, int32_t* idx,
                                   void* ws, size_t ws_bytes, void* stream);
/* Fused Communicator.step for TopK + ResidualMemory (grace_dl/dist/__init__.py:47-51):
 *   t = beta*r + gamma*g (t = g when has_residual == 0), payload = topk(t), r <- t - decode(payload)
 *   out (may be NULL): the world-1 Allgather result, zeros with t scattered at the payload.
 * `residual` is updated in place (it may hold garbage when has_residual == 0). */
grace_status_t grace_topk_residual_step(const float* g, float* residual, int32_t has_residual,
                                        float beta, float gamma, int64_t n, int64_t k, float* vals,
                                        int32_t* idx, float* out, void* ws, size_t ws_bytes,
                                        void* stream);
/* zeros(n).scatter_(idx, vals)  (topk.py:45-49; threshold.py:25-26; randomk.py:39-40). */
grace_status_t grace_sparse_decode(const float* vals, const int32_t* idx, int64_t count, float* out,
                                   int64_t n, void* stream);
grace_status_t grace_sparse_decode_i64(const float* vals, const int64_t* idx, int64_t count,
                                       float* out, int64_t n, void* stream);
/* Decode + aggregate of W gathered sparse payloads, exactly ((0 + d_0) + d_1 + ...) / divisor in
 * rank order (allgather.py:40-45).  vals/idx are rank-major [world][stride]; counts_host[w] is
 * rank w's payload length.  tags is an int32[n] scratch array (no initialisation needed). */
grace_status_t grace_sparse_aggregate(const float* vals, const int32_t* idx, int64_t stride,
                                      const int64_t* counts_host, int32_t world, float divisor,
                                      float* out, int32_t* tags, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GRACE_HIP_H */

/*
 * athd - C ABI of the MI355X-native AudioTextHTDemucs hot path (libathd.so).
 *
 * Replaces, for the per-segment inference path, the reference's Python surface:
 *   AudioTextHTDemucs(htdemucs, clap, tokenizer)          /root/reference/src/models/stem_separation/ATHTDemucs_v2.py:151-188
 *   model.load_state_dict(ckpt["model_state_dict"], strict=False)   test_inference.py:34-35
 *   model.forward(wav, text) -> (B,2,T)                   ATHTDemucs_v2.py:250-326
 * The CLAP text tower (ATHTDemucs_v2.py:238-248) stays on the host side: callers pass prompt embeddings
 * (B x 512 or P x 512 fp32, L2-normalised as ClapModel.get_text_features returns them).
 *
 * Conventions: plain pointers and sizes, no torch types.  All device pointers are HIP device memory owned by
 * the caller (wav, text embeddings, output, workspace); the context owns the packed weights.  Every call
 * returns 0 on success or a negative athd_status; the message is in athd_last_error().  Nothing is thrown
 * across the ABI.  Work is enqueued on the caller's stream (a hipStream_t passed as void*, NULL = default
 * stream); athd_forward* do not synchronise the host and create no memory, streams or events (the time branch's
 * stream and the fork/join events are made by athd_finalize), so they can be captured in a graph.  One context
 * per device; calls on one context must be serialised by the caller, even from different streams (the fork/join
 * events are per context).
 */
#ifndef ATHD_H
#define ATHD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct athd_ctx athd_ctx;

enum athd_status {
    ATHD_OK = 0,
    ATHD_EINVAL = -1,      /* bad argument / shape */
    ATHD_EKEY = -2,        /* unknown, missing or mis-shaped weight */
    ATHD_ESTATE = -3,      /* not finalized / already finalized */
    ATHD_EHIP = -4,        /* HIP runtime error */
    ATHD_EWORKSPACE = -5   /* workspace too small */
};

enum athd_dtype { ATHD_F32 = 0, ATHD_BF16 = 1 };

/* ABI version (major*100 + minor). */
int athd_version(void);

/* Create a context on HIP device `device`.  dtype: ATHD_F32 = exact fp32 MFMA everywhere (parity mode),
 * ATHD_BF16 = bf16 MFMA operands with fp32 accumulation/normalisation (throughput mode). */
int athd_create(athd_ctx** out, int device, int dtype);

/* Stage one weight tensor under its reference state-dict key (e.g. "htdemucs.encoder.0.conv.weight",
 * "text_attn.out_mlp.0.weight", "freq_decoder.layers.1.0.weight").  host points to contiguous fp32
 * (src_dtype 0) with the given shape.  Keys outside the hot path (clap.*, htdemucs.decoder.*, ...) are
 * accepted and ignored, mirroring load_state_dict(strict=False). */
int athd_set_weight(athd_ctx* ctx, const char* key, const void* host, const int64_t* shape, int ndim,
                    int src_dtype);

/* Number / names of the weight keys the hot path requires (reference names). */
int athd_num_required_keys(void);
const char* athd_required_key(int i);

/* Validate that every required key is present with the right shape, pack (transpose, tap-major, GLU pair
 * order, ConvTranspose residue split, bf16 conversion) and upload. */
int athd_finalize(athd_ctx* ctx);

/* (segment, prompt) items the decoder processes per chunk (default 64; 1..4096).  The encoder's buffers scale
 * with B and the decoder's with this setting: at B = 64, T = 264600 (6 s), P = 4 the workspace is about 18 GB
 * at 64 items and about 49 GB at 256 (the whole batch in one decode chunk: fewer, larger launches, the bench setting).
 * Takes effect for the next athd_workspace_bytes / athd_forward* calls; the environment variable
 * ATHD_DECODE_ITEMS overrides it. */
int athd_set_decode_items(athd_ctx* ctx, int64_t items);

/* Workspace bytes needed by athd_forward (P = 1) / athd_forward_prompts (P prompts) for B segments of
 * T samples (see athd_set_decode_items for the sizes at the bench configuration). */
size_t athd_workspace_bytes(athd_ctx* ctx, int64_t B, int64_t T, int P);

/* wav: (B,2,T) f32, text_emb: (B,512) f32 -> out: (B,2,T) f32.  == AudioTextHTDemucs.forward(wav, text). */
int athd_forward(athd_ctx* ctx, const float* wav, int64_t B, int64_t T, const float* text_emb, float* out,
                 void* workspace, size_t workspace_bytes, void* stream);

/* Encode once, decode once per prompt (1 <= P <= 256): wav (B,2,T), text_table (P,512) -> out (B,P,2,T); equal to P calls of
 * athd_forward because the encoder and cross-transformer do not see the prompt (ATHTDemucs_v2.py:278-283). */
int athd_forward_prompts(athd_ctx* ctx, const float* wav, int64_t B, int64_t T, const float* text_table, int P,
                         float* out, void* workspace, size_t workspace_bytes, void* stream);

/* ---- Track level: the window loop of test_inference.py:92-141 and sdr_loss (src/loss.py:9-30) ----
 * Windows: start_k = k*hop with hop = chunk_len - overlap, for k = 0 .. athd_num_windows()-1 (while start < length),
 * end_k = min(start_k + chunk_len, length).  Window k is faded by torchaudio Fade(fade_in = k ? overlap : 0,
 * fade_out = end_k < length ? overlap : 0, 'linear') and summed into the track in ascending k.  (The reference
 * fails when a window is shorter than its fade; callers check that with the plan.) */
int64_t athd_num_windows(int64_t length, int64_t chunk_len, int64_t overlap);

/* windows: device (k1-k0, n_stems, 2, chunk_len) f32, row k-k0 = model output of window k in its first
 * end_k - start_k samples.  out: device (n_stems, 2, end_{k1-1} - start_{k0}) f32, the track span of windows
 * [k0, k1) (the whole track for k0 = 0, k1 = athd_num_windows()).  Enqueued on `stream`. */
int athd_overlap_add(const float* windows, int64_t length, int64_t chunk_len, int64_t overlap, int n_stems,
                     int64_t k0, int64_t k1, float* out, void* stream);

/* ---- Track level, benchmark.py protocol (OurModel._chunked_inference, benchmark.py:155-204) ----
 * Same window starts (hop = chunk_len - overlap, while start < length); every window's model input is zero-padded
 * to chunk_len, its first len_k = end_k - start_k outputs are used.  fade_len_k = min(overlap, len_k / 2); the
 * window weight is 1 with linspace(0, 1, fade_len) over its first fade_len samples if start_k > 0 and
 * linspace(1, 0, fade_len) over its last fade_len samples if end_k < length; output += out_k * w and
 * weight += w in ascending k, then output / max(weight, 1e-8).
 * windows: device (k1-k0, n_stems, 2, chunk_len) f32.  weight == NULL: out (n_stems, 2, span) = the normalised
 * track span of windows [k0, k1) (the track itself for the full range).  weight != NULL (device, span floats):
 * out = the unnormalised sum and weight = the weight sum of the span, for sharded runs that add spans of window
 * ranges (the sum over ranks in rank order equals the single-range sum bit for bit) and then normalise with
 * athd_ola_normalize. */
int athd_overlap_add_weighted(const float* windows, int64_t length, int64_t chunk_len, int64_t overlap, int n_stems,
                              int64_t k0, int64_t k1, float* out, float* weight, void* stream);
/* out (rows, n) /= max(weight (n), 1e-8) in place (benchmark.py:201-202). */
int athd_ola_normalize(float* out, const float* weight, int rows, int64_t n, void* stream);

/* SDR of src/loss.py:9-30 with the sign of test_inference.py:153: est/target device (rows, n) f32 ->
 * *out (device f32) = mean over rows of clamp(10 log10((sum t^2 + 1e-8) / (sum (t-e)^2 + 1e-8)), -30, 30).
 * scratch: device, 2*rows doubles.  Sums are accumulated in fp64. */
int athd_sdr(const float* est, const float* target, int64_t rows, int64_t n, double* scratch, float* out,
             void* stream);

/* SI-SDR of src/loss.py:33-68 with the sign of benchmark.py:586: per row, zero-mean est e and target t,
 * a = <e,t> / (|t|^2 + 1e-8), clamp(10 log10((|a t|^2 + 1e-8) / (|e - a t|^2 + 1e-8)), -30, 30), mean over
 * rows -> *out (device f32).  scratch: device, 5*rows doubles.  fp64 sums. */
int athd_sisdr(const float* est, const float* target, int64_t rows, int64_t n, double* scratch, float* out,
               void* stream);

/* Kernel timing (measurement aid for bench.py; not part of the reference interface).  Between
 * athd_profile_start and athd_profile_stop every launch of kernel `kernel` (its rocprofv3 symbol without
 * "void athd::", the argument list and 'u' suffixes, e.g. "attn_bf16_kernel"; NULL or "" = all kernels) made
 * by this context's forwards is bracketed by HIP events on the launch stream.  athd_profile_stop synchronises
 * those events and aggregates per kernel: launches, summed event time, summed ALGORITHMIC flops and bytes.
 * kernel = "@section": every kernel, aggregated per forward section ("encoder", "transformer", "decoder").
 * kernel = "@sites": every kernel per call site, labelled "kernel@stage.site" (e.g.
 * "gemm4_kernel<129>@transformer.linear1"); kernel = "<kernel>@<stage.site>": every launch of that one call site.
 * While a profile is open the time branch runs on the caller's stream, so each event pair times one kernel. */
int athd_profile_start(athd_ctx* ctx, const char* kernel);
int athd_profile_stop(athd_ctx* ctx);
int athd_profile_count(athd_ctx* ctx);
int athd_profile_get(athd_ctx* ctx, int i, const char** kernel, long long* launches, double* ms, double* flops,
                     double* bytes);

/* Last error message of this context ("" if none). */
const char* athd_last_error(athd_ctx* ctx);

void athd_destroy(athd_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* ATHD_H */

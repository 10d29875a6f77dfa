/*
 * lfm_hip.h -- extern "C" HIP shim of the LFM predictor path (gfx950).
 *
 * This is the internal kernel boundary the host encoder (klb_imageIO) calls;
 * it replaces the reference's CUDA launchers and their call sites:
 *   predictorK_{tiles,angle,space}_GPU + symbolize_GPU
 *       (lfm_Predictors.h:16-40, called at klb_imageIO.cpp:1270-1300, :1696-1737)
 *       -> lfm_hip_predict  (all frames of a stack in one launch, fused symbolize)
 *   bwt_GPU + static_bwt_GPU + sum_bwt_GPU inside bwt_entropy_2D and the
 *   candidate loop of predict_and_2DEntropy / writeImage
 *       (lfm_Predictors.h:33-43; klb_imageIO.cpp:2030-2093, :2197-2225, :2273-2306)
 *       -> lfm_hip_select / lfm_hip_entropy2d
 *
 * Conventions: plain device pointers owned by the caller, explicit stream
 * (a hipStream_t passed as void*, NULL = default stream), asynchronous unless
 * stated, status code return.  The caller selects the device (hipSetDevice).
 */
#ifndef LFM_HIP_H
#define LFM_HIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum lfm_hip_status {
    LFM_HIP_OK = 0,
    LFM_HIP_EINVAL = 1,    /* bad argument                                   */
    LFM_HIP_ERUNTIME = 2,  /* HIP runtime error (launch / alloc / copy)      */
    LFM_HIP_ENOTINV = 3,   /* frame is not invertible (angle/space temporal) */
    LFM_HIP_ENODEV = 4     /* no usable GPU                                  */
};

/* families: 0 = tiles ("ANGLE_AND_SPACE", LFM_PREDICTOR_WAY 0), 1 = angle, 2 = space */

/* Forward predictor + symbolize for nframes consecutive frames of one volume.
 * d_in holds frames z0 .. z0+nframes-1 (W*H uint16 each, x fastest); frame
 * z is temporal when (video_bit & z) is odd, and then uses the raw frame z-1
 * (d_in of the previous frame, or d_prev for the first one).  predictor 0
 * copies the raw frames.  d_out receives uint16 symbols in the same layout. */
int lfm_hip_predict(const uint16_t* d_in, const uint16_t* d_prev, uint16_t* d_out, int W, int H, int nframes,
                    int T, int family, int predictor, int video_bit, int z0, void* stream);

/* Inverse of lfm_hip_predict (decode): symbols -> pixels for nframes frames
 * starting at global frame z0; a temporal first frame (video, odd z0) needs
 * the decoded frame z0-1 in d_prev.  ENOTINV for temporal frames of the
 * angle / space families (their residual is not invertible). */
int lfm_hip_unpredict(const uint16_t* d_sym, const uint16_t* d_prev, uint16_t* d_out, int W, int H, int nframes,
                      int T, int family, int predictor, int video_bit, int z0, void* stream);
/* lfm_hip_unpredict without the synchronisation: the kernels are queued on
 * `stream` and the launch's status word is copied into *h_status (pinned host
 * memory) behind them; once the stream has passed that point the caller hands
 * it to lfm_hip_unpredict_check.  The pipelined decode (gpu_decode) checks
 * each chunk's words at the event its download already waits for. */
int lfm_hip_unpredict_async(const uint16_t* d_sym, const uint16_t* d_prev, uint16_t* d_out, int W, int H,
                            int nframes, int T, int family, int predictor, int video_bit, int z0, int* h_status,
                            void* stream);
/* LFM_HIP_OK when a status word says the pixels are valid (0, or a band
 * hand-over timeout repaired on the device, reported on stderr), else
 * LFM_HIP_ERUNTIME. */
int lfm_hip_unpredict_check(int status);

/* The seven spatial candidates of one frame (predictors 1..7, symbolized) in
 * one launch: candidate k goes to d_out7 + (k-1)*W*H. */
int lfm_hip_predict_candidates(const uint16_t* d_frame, uint16_t* d_out7, int W, int H, int T, int family,
                               void* stream);

/* 2D entropy of a candidate buffer of npix uint16 symbols (450000-pixel
 * chunks, klb_imageIO.cpp:2030-2093).  Synchronous: writes the float result
 * (without the 0.96 raw-candidate factor) to *entropy. */
int lfm_hip_entropy2d(const uint16_t* d_cand, uint64_t npix, float* entropy, void* stream);

/* Predictor selection on one frame: builds the 8 candidates (0 = raw,
 * k = predictor k, spatial), their 2D entropies (candidate 0 scaled by 0.96)
 * and the reference argmin (exact ties -> highest index).  Synchronous.
 * d_workspace may be NULL (allocated internally) or hold
 * lfm_hip_select_workspace_bytes(W, H) bytes. */
size_t lfm_hip_select_workspace_bytes(int W, int H);
int lfm_hip_select(const uint16_t* d_frame, int W, int H, int T, int family, float entropy[8], int* chosen,
                   void* d_workspace, void* stream);

/* bzip2 (libbzip2 1.0.6 byte-exact) of the blocks [first, first + count) of
 * the x-fastest block grid of a device image (dims / bs as in the .lfm
 * header, bpp bytes per sample) at `level`: the compressed streams land
 * back to back in d_payload (block order); h_sizes[i] / h_flags[i] per
 * stream (flag != 0: the stream is NOT in the payload and must be produced by
 * the host library -- RLE1 block reaching nblockMAX, or a periodic block).
 * d_ws: lfm_hip_bzip2_workspace_bytes(count, blockBytes).  Synchronous. */
size_t lfm_hip_bzip2_workspace_bytes(uint32_t count, uint32_t block_bytes);
int lfm_hip_bzip2_blocks(const void* d_img, const uint32_t dims[5], const uint32_t bs[5], uint32_t bpp,
                         uint32_t first, uint32_t count, uint32_t level, void* d_ws, size_t ws_bytes,
                         void* d_payload, uint64_t* h_sizes, uint32_t* h_flags, void* stream);
/* Stage times (HIP events on its stream, ms) of the calling thread's last
 * lfm_hip_bzip2_blocks: [0] RLE1 + CRC, [1] BWT (buckets, chunk sorts, tie
 * rounds), [2] MTF + RUNA/RUNB, [3] Huffman tables, [4] bit emission +
 * compaction.  Returns 0, or 3 when no call has completed on this thread. */
int lfm_hip_bzip2_last_stage_ms(float ms[5]);
/* Progress hook of the calling thread's lfm_hip_bzip2_blocks calls: fn(ctx,
 * stage) once the device has finished stage 1 (BWT) and stage 2 (MTF + RUNA/
 * RUNB), at the host synchronisations that follow them, and stage 3 (the
 * Huffman tables; emission and compaction still queued behind them); fn ==
 * NULL removes it.  The pipelined encoder releases the next stack's GPU
 * bzip2 at stage 3 of each slot's last batch. */
void lfm_hip_bzip2_set_stage_hook(void (*fn)(void* ctx, int stage), void* ctx);

/* GPU bzip2 decode of `count` single-block streams (the .lfm block payloads,
 * SURVEY.md 8(f2); replaces the per-block BZ2_bzBuffToBuffDecompress of
 * klb_imageIO.cpp:1748-1821).  d_payload: device copy of the payload, 4-byte
 * aligned, readable 8 bytes past its end; stream i is h_offs[i] .. h_offs[i+1]
 * (host array of count + 1 byte offsets) and decodes into d_out + i *
 * out_stride.  h_lens[i] = decoded bytes; h_flags[i]: 0 ok, 1 decode this
 * stream with the host library (several blocks, randomised, malformed,
 * larger than out_stride), 2 block CRC mismatch.  d_ws:
 * lfm_hip_bunzip2_workspace_bytes(count, out_stride).  Synchronous. */
size_t lfm_hip_bunzip2_workspace_bytes(uint32_t count, uint32_t out_stride);
int lfm_hip_bunzip2_blocks(const void* d_payload, const uint64_t* h_offs, uint32_t count, void* d_out,
                           uint32_t out_stride, void* d_ws, size_t ws_bytes, uint32_t* h_lens, uint32_t* h_flags,
                           void* stream);
/* lfm_hip_bunzip2_blocks without the final synchronisation: returns once the
 * kernels and the copies into h_lens / h_flags are queued on `stream`
 * (h_lens / h_flags must be pinned host memory; read them after the stream or
 * an event recorded behind the call has completed).  The pipelined decode
 * (gpu_decode) overlaps one chunk's kernels with another's copies. */
int lfm_hip_bunzip2_issue(const void* d_payload, const uint64_t* h_offs, uint32_t count, void* d_out,
                          uint32_t out_stride, void* d_ws, size_t ws_bytes, uint32_t* h_lens, uint32_t* h_flags,
                          void* stream);

/* Decoded blocks first .. first + count - 1 (block i at d_blocks + (i -
 * first) * stride, x fastest) back into the device image (the inverse of the
 * writer's block gather, klb_imageIO.cpp:133-140).  Asynchronous. */
int lfm_hip_scatter_blocks(const void* d_blocks, uint32_t stride, uint32_t first, uint32_t count,
                           const uint32_t dims[5], const uint32_t bs[5], uint32_t bpp, void* d_img, void* stream);

/* Synthetic light-field stack of SURVEY.md 8(d) (integer generator) written
 * straight into device memory: frames z0 .. z0+Z-1 (X*Y pixels each) of
 * volume (c, t) = (0, t_index), global pixel index offset idx0 (a z-slab of a
 * c = t = 1 stack: z0 = first frame, idx0 = z0*X*Y). */
int lfm_hip_synth(uint16_t* d_out, int X, int Y, int Z, int T, int t_index, int z0, uint64_t idx0, uint64_t seed,
                  void* stream);

/* number of visible HIP devices (0 when no GPU / no runtime) */
int lfm_hip_device_count(void);

/* debug switch (env LFM_FORCE_GENERIC=1): route predictor launches to the
 * one-thread-per-pixel kernel instead of the LDS-ring kernel */
int lfm_hip_force_generic(void);

#ifdef __cplusplus
}
#endif
#endif

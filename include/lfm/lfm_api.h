/*
 * lfm_api.h -- liblfm extensions beyond the reference C ABI.
 *
 *  - lfm_set_family / lfm_get_family: the predictor family (0 tiles,
 *    1 angle, 2 space), a compile-time constant in the reference
 *    (src/common.h:19 LFM_PREDICTOR_WAY); default from env LFM_PREDICTOR_WAY.
 *  - writeLFMstack_c / readLFMstack_c: the MEX writeLFMstack / readLFMstack
 *    argument set (predictor request, Nnum, video flag) as plain C, for
 *    ctypes / cgo / JNI callers (matlabWrapper/writeLFMstack.cpp:360-433).
 *  - lfm_encoder_*: reusable encoder context that encodes to memory from a
 *    host or a DEVICE-resident stack and reports per-stage timings (bench).
 */
#ifndef LFM_API_H
#define LFM_API_H

#include <stdint.h>
#include <stddef.h>
#include "common.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LFM_API __attribute__((visibility("default")))

LFM_API int lfm_set_family(int family);
LFM_API int lfm_get_family(void);
/* Interface version of this header (also in lfm_version()'s string).
 * 2: lfm_decode_memory_roi takes out_bytes before numThreads (round 5; a
 *    caller built against version 1 passed numThreads third-to-last). */
#define LFM_API_VERSION 2
LFM_API const char* lfm_version(void);
LFM_API int lfm_api_version(void);

/* predictor_request: header bits 0-6 (0..7 auto, 8..15 forced k = request-8);
 * video: header bit 7.  Returns the writeKLBstack codes. */
LFM_API int writeLFMstack_c(const void* im, const char* filename, const uint32_t xyzct[KLB_DATA_DIMS],
                            int dataType, int numThreads, const float pixelSize[KLB_DATA_DIMS],
                            const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                            const char metadata[KLB_METADATA_SIZE], int predictor_request, int Nnum, int video);

/* Decode into im (caller-allocated, getImageSizeBytes); the header fields are
 * returned through the optional out pointers (headerVersion, Nnum). */
LFM_API int readLFMstack_c(const char* filename, void* im, int numThreads, uint8_t* headerVersion, uint8_t* Nnum);

typedef struct lfm_encode_stats {
    double total_ms;      /* whole encode, wall clock                        */
    double h2d_ms;        /* host -> device upload (0 for device input)      */
    double select_ms;     /* predictor selection (kernels + sync), wall       */
    double predict_ms;    /* predictor kernels, HIP events                    */
    double d2h_ms;        /* symbols device -> host                           */
    double compress_ms;   /* block compression + in-order assembly, wall      */
    int chosen;           /* predictor written to the header (bits 0-6)       */
    int header_version;   /* final header byte                                */
    float entropy[8];     /* candidate entropies when auto-selected, else 0   */
    uint64_t out_bytes;   /* size of the .lfm produced                        */
    double bz_stage_ms[5];/* GPU bzip2 stages (lfm_hip_bzip2_last_stage_ms order), HIP events,
                             summed over a HIP stream's batches, max over the streams */
    uint64_t bz_in_bytes; /* block bytes the GPU bzip2 stage compressed       */
} lfm_encode_stats;

typedef struct lfm_encoder lfm_encoder;

/* device < 0: current device; numThreads <= 0: host CPU share */
LFM_API lfm_encoder* lfm_encoder_create(int device, int numThreads);
LFM_API void lfm_encoder_destroy(lfm_encoder* enc);

/* Encode a stack to an in-memory .lfm.  img_is_device != 0: `img` is a device
 * pointer on the encoder's device.  *out stays valid until the next call on
 * this encoder or its destruction. */
LFM_API int lfm_encoder_encode(lfm_encoder* enc, const void* img, int img_is_device,
                               const uint32_t xyzct[KLB_DATA_DIMS], int dataType, int headerVersion, int Nnum,
                               const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                               const char metadata[KLB_METADATA_SIZE], const uint8_t** out, uint64_t* out_len,
                               lfm_encode_stats* stats);

/* Pipelined encode of a stack (z0 = 0, prev_frame = NULL) or of a z-slab
 * (arguments as lfm_encoder_encode_slab).  An auto request (headerVersion &
 * 0x7F < 8) on a slab with z0 > 0 returns 3: use lfm_encoder_submit_select
 * with the stack's frame 0, or a forced request 8 + k.  Runs the predictor stage (img may
 * be released on return), then hands the GPU bzip2 stage, the .lfm assembly
 * and its payload copies (system DMA engine) to a finisher thread and
 * returns.  The next submit's GPU bzip2 starts once this encode's kernels are
 * done (its selection and predictor stage run before, beside this one).  At
 * most two encodes are in flight: a submit first joins the one before last.
 * *ticket names the encode for lfm_encoder_wait; errors of the finisher are
 * returned by lfm_encoder_wait. */
LFM_API int lfm_encoder_submit(lfm_encoder* enc, const void* img, int img_is_device, const void* prev_frame,
                               uint32_t z0, const uint32_t xyzct[KLB_DATA_DIMS], int dataType, int headerVersion,
                               int Nnum, const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                               const char metadata[KLB_METADATA_SIZE], uint64_t* ticket);
/* lfm_encoder_submit with the frame auto-selection runs on: select_frame
 * (X*Y samples, host or device like img) is the whole stack's frame 0 when img
 * is a z-slab of it (z0 > 0), so every slab selects what the whole-stack
 * encode selects (klb_imageIO.cpp:2316-2360); NULL = img's own frame 0.  An
 * auto request (headerVersion & 0x7F < 8) on a slab with z0 > 0 needs it
 * (returns 3 otherwise).  Selection then runs inside the submit, on the
 * encoder's high-priority stream, after the previous encode's kernels. */
LFM_API int lfm_encoder_submit_select(lfm_encoder* enc, const void* img, int img_is_device, const void* prev_frame,
                                      uint32_t z0, const void* select_frame, const uint32_t xyzct[KLB_DATA_DIMS],
                                      int dataType, int headerVersion, int Nnum,
                                      const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                      const char metadata[KLB_METADATA_SIZE], uint64_t* ticket);
/* Wait for a submitted encode.  *out stays valid until the second submit
 * after it (or a synchronous encode on this encoder); returns its status.
 * On a nonzero status *out = NULL and *out_len = 0; 8 = the ticket was never
 * submitted on this encoder or its buffer set has been reused since. */
LFM_API int lfm_encoder_wait(lfm_encoder* enc, uint64_t ticket, const uint8_t** out, uint64_t* out_len,
                             lfm_encode_stats* stats);

/* Encode z-slab [z0, z0 + xyzct[2]) of a larger stack (c = t = 1) for
 * multi-GPU sharding: frame z of the slab is temporal when video & (z0 + z)
 * is odd, and the slab's first frame then uses prev_frame (the raw frame
 * z0 - 1, host or device like img).  Use a forced predictor request (8 + k,
 * k selected on the whole stack's frame 0) so every slab codes like the
 * whole stack would; slab depths must be multiples of the block depth except
 * the last.  The result is a valid .lfm of the slab (lfm_merge_slabs joins
 * them).  An auto request (headerVersion & 0x7F < 8) with z0 > 0 returns 3:
 * the slab's own frame 0 is not the stack's, so it cannot select what the
 * whole-stack encode selects. */
LFM_API int lfm_encoder_encode_slab(lfm_encoder* enc, const void* img, int img_is_device, const void* prev_frame,
                                    uint32_t z0, const uint32_t xyzct[KLB_DATA_DIMS], int dataType,
                                    int headerVersion, int Nnum, const uint32_t blockSize[KLB_DATA_DIMS],
                                    int compressionType, const char metadata[KLB_METADATA_SIZE],
                                    const uint8_t** out, uint64_t* out_len, lfm_encode_stats* stats);

/* Join the .lfm files of consecutive z-slabs into the whole stack's .lfm
 * (byte-identical to encoding the stack in one piece).  *out is malloc'ed:
 * release it with lfm_free.  Returns 0, or 3 when the slabs do not fit. */
LFM_API int lfm_merge_slabs(const uint8_t* const* slabs, const uint64_t* lens, int nslabs, uint8_t** out,
                            uint64_t* out_len);
LFM_API void lfm_free(void* p);

/* Multi-process writers (one process per GPU, e.g. torchrun): each rank
 * places its own z-slab .lfm into the whole stack's .lfm buffer `dst`
 * (shared memory), concurrently with the other ranks.  lfm_slab_info gives a
 * slab's payload bytes and block count (the values the ranks exchange);
 * lfm_place_slab copies the slab's payload to payload_offset (payload bytes
 * of the slabs before it), writes its block end offsets re-based into the
 * table at block_index (blocks before it) and, for block_index 0, the fixed
 * header with the stack's depth total_z.  The result equals lfm_merge_slabs. */
LFM_API int lfm_slab_info(const uint8_t* slab, uint64_t len, uint64_t* payload_bytes, uint64_t* nblocks);
LFM_API int lfm_place_slab(const uint8_t* slab, uint64_t slab_len, uint8_t* dst, uint64_t dst_len, uint32_t total_z,
                           uint64_t total_blocks, uint64_t block_index, uint64_t payload_offset, int numThreads);

/* Devices the writers farm block ranges to (klb_imageIO::writeImage,
 * writeKLBstack, writeLFMstack_c, lfm_encoder_encode_multi): n > 0 sets the
 * list (a device may repeat: several workers on one GPU); n = 0 restores the
 * default: env LFM_GPUS = "0,1,.." or a count; else, in a multi-process job,
 * one device when several processes share this node (LOCAL_WORLD_SIZE or
 * OMPI_COMM_WORLD_LOCAL_SIZE > 1, or only WORLD_SIZE > 1 known): LOCAL_RANK
 * (OMPI_COMM_WORLD_LOCAL_RANK) modulo the visible devices, the current device
 * when no local rank is set; else (one process on the node) every visible
 * device.  lfm_get_devices returns the count and fills up to cap entries. */
LFM_API int lfm_set_devices(const int* devices, int n);
LFM_API int lfm_get_devices(int* devices, int cap);
/* The default list above for n_visible devices and current device `current`
 * (no device call; what lfm_get_devices gives after lfm_set_devices(NULL, 0)
 * on such a machine).  Returns the count and fills up to cap entries. */
LFM_API int lfm_default_devices(int n_visible, int current, int* devices, int cap);

/* Encode a HOST stack on the device list above (one host thread per device,
 * block-layer ranges: z-slabs, or ranges of c / t), into the encoder's
 * in-memory .lfm (byte-identical to a one-device encode).  Falls back to the
 * encoder's own device when the list has one device or the stack one range. */
LFM_API int lfm_encoder_encode_multi(lfm_encoder* enc, const void* img, const uint32_t xyzct[KLB_DATA_DIMS],
                                     int dataType, int headerVersion, int Nnum,
                                     const uint32_t blockSize[KLB_DATA_DIMS], int compressionType,
                                     const char metadata[KLB_METADATA_SIZE], const uint8_t** out, uint64_t* out_len,
                                     lfm_encode_stats* stats);

/* Free the device / pinned buffers the writers keep between calls. */
LFM_API void lfm_release_encoders(void);

/* Decode an in-memory .lfm into `img` (host, getImageSizeBytes bytes). */
LFM_API int lfm_decode_memory(const uint8_t* buf, uint64_t len, void* img, int numThreads);
/* Decode the region lb .. ub (inclusive, xyzct) of an in-memory .lfm into
 * `out` (host, x fastest, out_bytes long): readKLBroiInPlace on memory.
 * Only the blocks the region depends on are decoded.  Returns 3 when the
 * region lies outside the image or out_bytes is less than the region's
 * pixels times the file's bytes per pixel (the header's data type). */
LFM_API int lfm_decode_memory_roi(const uint8_t* buf, uint64_t len, const uint32_t lb[KLB_DATA_DIMS],
                                  const uint32_t ub[KLB_DATA_DIMS], void* out, uint64_t out_bytes, int numThreads);

#ifdef __cplusplus
}
#endif
#endif

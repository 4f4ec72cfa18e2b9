/*
 * nfec.h -- C ABI of the MI355X-native NORM FEC engine (libnfec.so).
 *
 * Drop-in boundary for NORM's FEC plugin layer (reference include/normEncoder.h:38-54):
 * plain pointers, sizes and integer status codes; no C++ or torch types cross it.
 * Every compute entry point runs hand-written gfx950 HIP kernels (a missing/failed GPU yields
 * NFEC_EDEVICE; nothing falls back to the CPU), except the per-call entry points named *_host
 * ("host CPU per-call paths" below), which are the host path by definition: one Encode call of
 * NORM's incremental sender, or one block's repair, is microseconds of work, less than a GPU
 * round trip.  Which of the two a drop-in class calls is its documented policy, not a fallback.
 *
 * Reference interfaces each entry replaces (paths in USNavalResearchLaboratory/norm):
 *   nfec_codec_create(_ex) NormEncoderRS8::Init  src/common/normEncoderRS8.cpp:400-462
 *                         NormDecoderRS8::Init   src/common/normEncoderRS8.cpp:542-649
 *                         NormEncoderRS16::Init  src/common/normEncoderRS16.cpp:399-461
 *                         NormEncoderMDP::Init   src/common/normEncoderMDP.cpp:56-84
 *   nfec_codec_destroy    NormEncoderXX::Destroy / NormDecoderXX::Destroy (e.g. normEncoderRS8.cpp:464-471)
 *   nfec_encode           the per-segment NormEncoder::Encode loop as run by
 *                         NormObject::CalculateBlockParity  src/common/normObject.cpp:2203-2229
 *                         (NormEncoderRS8::Encode normEncoderRS8.cpp:473-483, RS16 :472-482,
 *                          MDP normEncoderMDP.cpp:178-211) for many blocks at once
 *   nfec_decode           NormDecoder::Decode  (RS8 normEncoderRS8.cpp:652-757, RS16 :650-755,
 *                         MDP normEncoderMDP.cpp:333-430) for many blocks at once, as called
 *                         from NormObject::HandleObjectMessage src/common/normObject.cpp:1548-1644
 *   nfec_encode_host_vectors / nfec_decode_host_vectors
 *                         the same two sites on NORM's scattered segment lists (block->SegmentList())
 *   nfec_encode_segment   NormEncoder::Encode(segmentId, dataVector, parityVectorList)
 *                         (include/normEncoder.h:44), host pointers, exact per-call semantics
 *   nfec_decode_vectors   NormDecoder::Decode(vectorList, numData, erasureCount, erasureLocs)
 *                         (include/normEncoder.h:53), host pointers, exact per-call semantics
 *   nfec_encode_segment_host / nfec_decode_vectors_host
 *                         the same two calls on the host CPU (GFNI / AVX2 region products)
 */
#ifndef NFEC_H
#define NFEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NFEC_ABI_VERSION 1

/* codec families (NORM fec_id 5/2 -> RS8/RS16, fec_id 129 -> MDP; normSession.cpp:839-875) */
enum {
    NFEC_RS8 = 1,  /* GF(2^8) systematic Reed-Solomon, Rizzo Vandermonde generator   */
    NFEC_RS16 = 2, /* GF(2^16) systematic Reed-Solomon, native-endian 16-bit symbols */
    NFEC_MDP = 3   /* legacy GF(2^8) LFSR code (fec_id 129)                          */
};

/* status codes: >= 0 success */
enum {
    NFEC_OK = 0,
    NFEC_EINVAL = -1,   /* bad argument (sizes, alignment, null pointers)            */
    NFEC_ENOMEM = -2,   /* device or host allocation failed                            */
    NFEC_EDEVICE = -3,  /* HIP runtime/launch failure or no usable gfx950 device       */
    NFEC_ERANGE = -4,   /* numData + numParity exceeds the field (Init returns false)  */
    NFEC_ENOTSUP = -5   /* combination not supported (e.g. accumulate with MDP encode) */
};

/* batch flags */
enum {
    /* XOR results into the existing output bytes, exactly like the reference's
     * accumulate-into-caller-zeroed-buffer contract (Encode parity, Decode erased
     * source).  Without it outputs are overwritten, which is byte-identical whenever
     * the caller zeroed them first (NORM always does: normObject.cpp:1579, :2240-2252). */
    NFEC_ACCUMULATE = 1u << 0
};

typedef struct nfec_codec nfec_codec;

typedef struct nfec_codec_info {
    int32_t kind;         /* NFEC_RS8 / NFEC_RS16 / NFEC_MDP */
    int32_t device;       /* HIP device ordinal the codec lives on (-1: host-only codec) */
    uint32_t num_data;    /* k (ndata)  */
    uint32_t num_parity;  /* m (npar)   */
    uint32_t vector_size; /* bytes per segment vector processed (vectorSize given to Init) */
    uint32_t symbol_bytes;/* 1 (RS8/MDP) or 2 (RS16) */
} nfec_codec_info;

/*
 * A batch of FEC blocks resident in device memory (HBM).
 * Block b, segment slot s starts at  blocks + b*block_stride + s*seg_stride.
 * Slot layout per block mirrors NORM's block segment list (normSegment.h:79,
 * normObject.cpp:1610): slots [0, numData) hold source symbols, slots
 * [numData, numData + m) hold parity symbols.
 * Requirements: blocks, seg_stride and block_stride are multiples of 8 bytes
 * (NORM's segment pool is 8-byte aligned, normSegment.cpp:25-27), and
 * seg_stride >= vector_size.
 */
typedef struct nfec_block_batch {
    void* blocks;              /* device pointer */
    uint64_t block_stride;     /* bytes */
    uint32_t seg_stride;       /* bytes */
    uint32_t nblocks;
    const uint16_t* num_data;  /* device [nblocks] per-block numData (<= k), or NULL = k */
    uint32_t flags;            /* NFEC_ACCUMULATE */
    uint32_t reserved;
} nfec_block_batch;

/* ---- version / device ---- */
int nfec_abi_version(void);
/* SHA-256 (hex) of the sources this library was built from: the .cpp/.hip/.hpp/.h files of
 * norm_amd/csrc, then the .h files of include and include/norm_fec, each list sorted by path,
 * contents concatenated (norm_amd/Makefile). */
const char* nfec_build_id(void);
/* number of visible gfx950 devices (0 when none) */
int nfec_device_count(void);
/* human-readable message for the last error on this thread */
const char* nfec_last_error(void);

/* ---- host-only generator construction (no GPU needed) ----
 * Writes the m x k parity rows of the systematic generator (RS8/RS16: Rizzo Vandermonde
 * code, normEncoderRS8.cpp:428-450; MDP: the LFSR block map for k source symbols),
 * row-major, symbol_bytes per element.  Returns NFEC_ERANGE where Init would return false. */
int nfec_build_generator(int kind, uint32_t num_data, uint32_t num_parity, void* host_out, size_t bytes);

/* ---- codec lifecycle ---- */
int nfec_codec_create(int device, int kind, uint32_t num_data, uint32_t num_parity,
                      uint32_t vector_size, nfec_codec** out);

/* Codec options (nfec_codec_config.flags): correct alternatives of the RS16 kernels, chosen per
 * codec (the tests run both; the defaults are the faster ones), and a codec without a GPU. */
enum {
    NFEC_OPT_RS16_SHARED_TABLES = 1u << 0, /* RS16 products on the shared-LDS-table kernel
                                              instead of the tower-field one */
    NFEC_OPT_RS16_TOEPLITZ_OFF = 1u << 1,  /* RS16 encode never uses the Toeplitz split */
    NFEC_OPT_RS16_TOEPLITZ_ON = 1u << 2,   /* ... uses it whenever the shape allows it, not
                                              only where it needs fewer passes */
    NFEC_OPT_HOST_ONLY = 1u << 3,          /* no device at all (a NORM node without a usable
                                              gfx950): Init's math on the host, and only the host
                                              per-call paths (nfec_encode_segment_host,
                                              nfec_decode_vectors_host) run; every GPU entry
                                              returns NFEC_EDEVICE.  No device list. */
    NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL = 1u << 4  /* the Toeplitz split at one Karatsuba level at
                                                   most (default: two where they save passes) */
};

/* One codec over one or several GPUs of a node.  With several devices the codec holds the
 * generator on each (one full codec per device; a device may be listed twice, which gives two
 * independent pipelines on it) and stripes every host batch (nfec_*_host, nfec_*_host_vectors
 * and their async forms) over them in contiguous block ranges [i*B/N, (i+1)*B/N), one host
 * thread and one staging pipeline per device, no exchange between the ranges: the in-process
 * form of SURVEY 8e's block striping for single-process callers such as one NORM session
 * (normSession.cpp:834-889) or npc (normPrecode.cpp:588-880).  A device batch (nfec_encode /
 * nfec_decode) runs on the first listed device that holds it (NFEC_EINVAL when a device
 * allocation is on none of them; a batch in host-mapped or registered host memory runs on the
 * first device, as a one-device codec would take it);
 * per-call work (nfec_encode_segment / nfec_decode_vectors) on the first device. */
typedef struct nfec_codec_config {
    int32_t kind;             /* NFEC_RS8 / NFEC_RS16 / NFEC_MDP */
    uint32_t num_data, num_parity, vector_size;
    const int32_t* devices;   /* HIP device ordinals (NULL with num_devices 0: device 0) */
    uint32_t num_devices;     /* 0 or 1: one device; at most 64 */
    uint32_t flags;           /* NFEC_OPT_* */
} nfec_codec_config;
int nfec_codec_create_ex(const nfec_codec_config* config, nfec_codec** out);
/* Number of devices of a codec; their ordinals go to devices[0 .. min(n, cap)) when non-NULL. */
int nfec_codec_num_devices(const nfec_codec* codec, int32_t* devices, uint32_t cap);
void nfec_codec_destroy(nfec_codec* codec);
int nfec_codec_get_info(const nfec_codec* codec, nfec_codec_info* out);
/* Encode paths the codec chose at creation (bit mask, < 0 on error):
 *   NFEC_FEATURE_RS16_TOEPLITZ: unshortened, overwriting RS16 encodes use the Toeplitz split of
 *   the generator (three (m/2)-row products over k/2 columns). */
#define NFEC_FEATURE_RS16_TOEPLITZ 1
/* ... at two Karatsuba levels: nine (m/4)-row products over k/4 columns (tower kernel) */
#define NFEC_FEATURE_RS16_TOEPLITZ2 2
int nfec_codec_features(const nfec_codec* codec);
/* Device-batch encodes so far per path that took them (diagnostics: which kernel family a
 * batch shape reaches).  counts[i] for i < n; returns NFEC_PATH_COUNT (< 0 on error). */
#define NFEC_PATH_FIXED 0        /* bit-sliced kernels generated for the (k, m) generator (RS8, MDP; shortened RS8 too) */
#define NFEC_PATH_RUNTIME 1      /* bit-sliced, runtime coefficients (any RS8 / MDP shape) */
#define NFEC_PATH_RS16_SPLIT 2   /* RS16 Toeplitz split (shortened batches too, tower kernel) */
#define NFEC_PATH_RS16_PRODUCT 3 /* RS16 one product over all k columns (tower or shared-table kernel) */
#define NFEC_PATH_GENERIC 4      /* table-lookup kernels */
#define NFEC_PATH_COUNT 5
int nfec_codec_encode_paths(const nfec_codec* codec, uint64_t* counts, uint32_t n);
/* The same for device-batch decodes (NFEC_DPATH_*). */
#define NFEC_DPATH_FIXED 0        /* RS8 closed-form plan + fused / bit-sliced repair for the (k, m) generator (shortened too) */
#define NFEC_DPATH_RUNTIME 1      /* one-pass repair on the runtime-coefficient kernel (any RS8 shape, MDP) */
#define NFEC_DPATH_RS16_TOWER 2   /* RS16 closed-form plan, both stages on the tower kernel */
#define NFEC_DPATH_GENERIC 3      /* Gauss-Jordan plan and table-lookup kernels */
#define NFEC_DPATH_COUNT 4
int nfec_codec_decode_paths(const nfec_codec* codec, uint64_t* counts, uint32_t n);
/* Copies the m x k parity rows of the systematic generator (row p = generator row k+p),
 * row-major, elements of symbol_bytes each.  MDP: the m x k matrix of the LFSR code for a
 * full block of k source symbols.  bytes must be >= m*k*symbol_bytes. */
int nfec_codec_get_generator(const nfec_codec* codec, void* host_out, size_t bytes);

/* ---- batched device-resident path (the performance path) ----
 * stream is a hipStream_t (NULL = legacy default stream).  Calls are asynchronous with
 * respect to the host; results are ready when the stream reaches them.  (A large RS16 encode on
 * the two-level Toeplitz split runs half of its sub-batches on a second stream of the codec's
 * own; that stream starts after the caller's stream and joins it before the call's end, so the
 * ordering the caller sees is the same.) */
int nfec_encode(nfec_codec* codec, const nfec_block_batch* batch, void* stream);

/* erasure_locs: device [nblocks][erasure_stride] sorted slot indices (source erasures
 * first, then missing parity, as NormObject builds them); erasure_counts: device
 * [nblocks]; status: device [nblocks] or NULL -- per block the reference Decode return
 * value (erasureCount on success, 0 when the block cannot be repaired).
 * Erased source slots are repaired; parity slots are never written.
 * A codec owns one decode workspace (like the reference decoder's scratch matrices,
 * normEncoderRS8.cpp:559-606): decode calls on one codec must be ordered (same stream, or
 * synchronised by the caller); encode calls only read the codec and may run concurrently. */
int nfec_decode(nfec_codec* codec, const nfec_block_batch* batch, const uint16_t* erasure_locs,
                uint32_t erasure_stride, const uint16_t* erasure_counts, int32_t* status,
                void* stream);

/* ---- host-resident batched path: same layouts, host pointers (pageable or pinned).
 * Staged through pinned buffers with H2D / compute / D2H overlapped on streams.
 * Synchronous: returns when all outputs are back in host memory.  A codec owns one staging
 * pipeline: host-batch calls (these and the *_host_vectors calls) on one codec from several
 * host threads are serialised; calls on different codecs run concurrently. */
int nfec_encode_host(nfec_codec* codec, const nfec_block_batch* host_batch);
int nfec_decode_host(nfec_codec* codec, const nfec_block_batch* host_batch,
                     const uint16_t* erasure_locs, uint32_t erasure_stride,
                     const uint16_t* erasure_counts, int32_t* status);

/* ---- host segment lists: many blocks, each a list of scattered segment pointers ----
 * The batch form of NormObject::CalculateBlockParity (src/common/normObject.cpp:2203-2229)
 * and of the receiver's NormSenderNode::Decode site (normObject.cpp:1548-1644), where a
 * block is block->SegmentList(): pointers into NORM's segment pool (normSegment.cpp:14-86).
 * vectors[b*(k+m) + s] is block b's slot s: slots [0, numData_b) source, [numData_b,
 * numData_b + m) parity; each holds >= vector_size bytes.  num_data: host [nblocks] or NULL
 * (= k).  Encode writes the parity vectors (XOR into them with NFEC_ACCUMULATE).  Decode
 * writes only the erased source vectors listed in erasure_locs[b*erasure_stride ..] (sorted,
 * erasure_counts[b] entries); parity pointers may be NULL (absent, never dereferenced;
 * MDP reads them as zero).  status (host [nblocks], may be NULL) as nfec_decode.  RS16 never
 * writes an odd last byte.  Synchronous; segments are gathered into pinned staging by host
 * threads, with H2D / compute / D2H overlapped. */
int nfec_encode_host_vectors(nfec_codec* codec, void* const* vectors, uint32_t nblocks,
                             const uint16_t* num_data, uint32_t flags);
int nfec_decode_host_vectors(nfec_codec* codec, void* const* vectors, uint32_t nblocks,
                             const uint16_t* num_data, const uint16_t* erasure_locs,
                             uint32_t erasure_stride, const uint16_t* erasure_counts,
                             int32_t* status, uint32_t flags);

/* ---- asynchronous segment-list batches: receiver-side cross-block batching ----
 * The receiver's decode site (NormObject::HandleObjectMessage -> NormSenderNode::Decode,
 * normObject.cpp:1548-1644, normNode.h:484-487) runs one block per call on NORM's protocol
 * thread.  These queue a batch of blocks on the codec and return at once; the protocol thread
 * keeps receiving and later collects the completion.  Arguments as the synchronous calls; the
 * pointer table, num_data, erasure lists and counts are copied at submission, the segment
 * buffers and the status array must stay valid until the request completes.  A codec runs its
 * requests in submission order on a worker thread of its own; different codecs (one decoder
 * per remote sender, normNode.h:649) run concurrently.  Destroying a codec completes its
 * queued requests first (their handles must still be waited on or were already). */
typedef struct nfec_request nfec_request;
int nfec_encode_host_vectors_async(nfec_codec* codec, void* const* vectors, uint32_t nblocks,
                                   const uint16_t* num_data, uint32_t flags, nfec_request** request);
int nfec_decode_host_vectors_async(nfec_codec* codec, void* const* vectors, uint32_t nblocks,
                                   const uint16_t* num_data, const uint16_t* erasure_locs,
                                   uint32_t erasure_stride, const uint16_t* erasure_counts,
                                   int32_t* status, uint32_t flags, nfec_request** request);
/* 1 when the request has completed, 0 while pending (non-blocking poll). */
int nfec_request_test(nfec_request* request);
/* Blocks until completion, frees the request and returns the call's status code. */
int nfec_request_wait(nfec_request* request);

/* ---- per-call NORM semantics with scattered host vectors (drop-in classes) ---- */
/* NormEncoder::Encode: parity_vectors[i] ^= G[k+i][segment_id] * data over vector_size
 * bytes (RS16: vector_size/2 symbols).  MDP: one in-order LFSR step. Synchronous. */
int nfec_encode_segment(nfec_codec* codec, uint32_t segment_id, const void* data,
                        void* const* parity_vectors);
/* NormDecoder::Decode: returns erasure_count on success, 0 when undecodable, <0 on error. */
int nfec_decode_vectors(nfec_codec* codec, void* const* vector_list, uint32_t num_data,
                        uint32_t erasure_count, const uint32_t* erasure_locs);
/* ---- host CPU per-call paths (NORM's incremental sender, one-block repair) ----
 * NormObject::NextSenderMsg calls Encode once per source segment and reads the parity without
 * a call that ends the block (normObject.cpp:2038-2052), so each call must finish on return:
 * m products of one segment, microseconds of CPU work against ~80 us for a GPU round trip
 * (INTEGRATION.md section 1).  These run on the calling CPU thread: GF(2^8) products by GFNI
 * affine transforms, AVX2 nibble tables or a scalar product table, whichever the CPU has. */
enum { NFEC_HOST_GF_SCALAR = 0, NFEC_HOST_GF_AVX2 = 1, NFEC_HOST_GF_GFNI = 2 };
/* dst[0..bytes) ^= c * src[0..bytes) in the RS8 field (0x11d).  isa: an NFEC_HOST_GF_* form, or
 * < 0 for the best this CPU has.  Returns the form used, NFEC_ENOTSUP when the CPU lacks it. */
int nfec_gf8_addmul_host(void* dst, const void* src, uint8_t c, size_t bytes, int isa);
/* ... over `symbols` native-endian 16-bit symbols in the RS16 field (0x1100B); forms: GFNI or
 * scalar (an AVX2 request runs the scalar form, which is what it returns). */
int nfec_gf16_addmul_host(void* dst, const void* src, uint16_t c, size_t symbols, int isa);
/* Row dot product, the body of nfec_decode_vectors_host:
 *   dst[0..n) = (accumulate ? dst : 0) + sum_j coef[j] * src[j][0..n)
 * over n bytes (bits = 8, RS8 / MDP field) or n native-endian symbols (bits = 16, RS16 field),
 * one pass over dst.  Returns the form used (as above), NFEC_EINVAL / NFEC_ENOTSUP otherwise. */
int nfec_gf_dot_host(int bits, void* dst, const void* const* src, const uint16_t* coef, uint32_t ncols,
                     size_t n, int accumulate, int isa);
/* NormEncoderRS8::Encode (normEncoderRS8.cpp:473-483) on the host: parity_vectors[i] ^=
 * G[k+i][segment_id] * data over vector_size bytes.  RS16 (NormEncoderRS16::Encode,
 * normEncoderRS16.cpp:472-482): the same over vector_size / 2 native-endian symbols, an odd last
 * byte untouched.  MDP (NormEncoderMDP::Encode, normEncoderMDP.cpp:178-211): one LFSR step,
 * s = data ^ parity[0], parity[i] = parity[i+1] ^ g[m-1-i] * s, parity[m-1] = g[0] * s --
 * segments in order, as the reference requires (segment_id is ignored, as there).  Reads only
 * the codec's generator: concurrent calls on one codec are safe (on different blocks). */
int nfec_encode_segment_host(nfec_codec* codec, uint32_t segment_id, const void* data,
                             void* const* parity_vectors);

/* NormDecoderRS8::Decode / NormDecoderRS16::Decode (normEncoderRS8.cpp:652-757, RS16 :650-755)
 * and NormDecoderMDP::Decode (normEncoderMDP.cpp:333-430) on the host CPU, same contract as
 * nfec_decode_vectors.  RS: the block's closed-form repair map (the first surviving parities
 * substitute for the erased source, rs8_plan_rt_kernel's algebra) applied with the GFNI / AVX2
 * region products, XORed into the erased source buffers.  MDP: the closed-form Forney map
 * (mdp_plan_kernel's) over the surviving slots, written over the erased source.  Returns
 * erasure_count, 0 when undecodable or the list is not sorted / in range (block untouched),
 * NFEC_ENOTSUP for RS16 codes past the closed form (min(k, m) > 64).  A one-block repair of a
 * NORM-sized block is tens of microseconds of CPU work, below the GPU round trip. */
int nfec_decode_vectors_host(nfec_codec* codec, void* const* vectors, uint32_t num_data,
                             uint32_t erasure_count, const uint32_t* erasure_locs);
/* 1 when nfec_decode_vectors_host is the faster path for this call, else 0 (the drop-in
 * Decode's choice), from the measured latencies: RS8 while erasures x numData x vector bytes
 * stays within 256 MiB, MDP while erasures x (numData + numParity) x vector bytes stays within
 * 512 MiB, RS16 (min(k, m) <= 64) while erasures x numData x symbols stays within 64 Mi. */
int nfec_decode_host_preferred(const nfec_codec* codec, uint32_t num_data, uint32_t erasure_count);

/* sizeof() of the drop-in class NormEncoder<kind> (decoder = 0) or NormDecoder<kind>
 * (decoder = 1) as the library was compiled (include/norm_fec/normEncoder*.h), 0 for an
 * unknown kind: a NORM build can check that its translation units see the same layout. */
size_t nfec_dropin_sizeof(int kind, int decoder);

/* The host worker pool every host-batch copy of 4 MiB or more runs on (one per process): its
 * workers (the cores the job may use -- the affinity mask capped by the cgroup cpu.max quota --
 * or NFEC_HOST_THREADS, at most 64), the usable and the visible cores.  All stripes of all codecs
 * share it; smaller copies run on the calling thread. */
int nfec_host_threads(uint32_t* pool, uint32_t* usable_cores, uint32_t* visible_cores);
/* Self-check of that pool (tests): runs `pieces` pieces on it.  mode 0: every piece counts once;
 * 1: piece 1 throws std::bad_alloc; 2: piece 1 throws std::runtime_error.  Returns the pieces that
 * ran to completion (mode 0: all of them), or the pool's error status (NFEC_ENOMEM / NFEC_EINVAL)
 * once every piece has run -- a throwing piece neither ends the process nor leaves the call
 * waiting.  Safe in a child forked after the pool started (its pieces then run inline). */
int nfec_util_pool_check(uint32_t pieces, int mode);
/* Host-side rate probe of the segment-list gather (no GPU): nstripes driver threads, one per
 * would-be device, each gather their contiguous block range [i*B/N, (i+1)*B/N) of the pointer
 * table vectors[b*slots + s] (slots vectors of vector_size bytes per block) into staging of their
 * own in the pipelines' 128 MiB chunks, through the same pool as nfec_*_host_vectors.  *seconds:
 * the mean wall time of one pass over all blocks; *max_active (may be NULL): the most copy
 * pieces that ran at once during the probe (at most the pool's size). */
int nfec_util_gather_probe(void* const* vectors, uint32_t nblocks, uint32_t slots, uint32_t vector_size,
                           uint32_t nstripes, uint32_t reps, double* seconds, uint32_t* max_active);
/* ---- synthetic workload utilities (device kernels; SURVEY.md 8d definitions) ----
 * fill: source slots [0, numData) of every block with the splitmix64 stream
 *       word w of (block b, slot s) = mix(seed ^ ((b0+b)<<20) ^ s + (w+1)*0x9E3779B97F4A7C15).
 * erasures: per block `count` sorted distinct indices in [0, range), Fisher-Yates over the
 *           counter stream mix(seed ^ 0xE7A5E7A500000000 ^ (b0+b) + (i+1)*gamma).
 * zero: zero the listed slots of every block (the receiver's zero-fill, normObject.cpp:1579).
 * stream_copy: device-to-device copy of `bytes` (16-byte aligned pointers and size) by a
 *       streaming kernel, for the bench's achievable-HBM-rate figure. */
int nfec_util_fill(const nfec_block_batch* batch, uint32_t num_data, uint32_t vector_size,
                   uint64_t seed, uint64_t first_block, void* stream);
int nfec_util_erasures(uint16_t* erasure_locs, uint32_t erasure_stride, uint16_t* erasure_counts,
                       uint32_t nblocks, uint32_t range, uint32_t count, uint64_t seed,
                       uint64_t first_block, void* stream);
int nfec_util_zero_slots(const nfec_block_batch* batch, const uint16_t* erasure_locs,
                         uint32_t erasure_stride, const uint16_t* erasure_counts,
                         uint32_t vector_size, void* stream);
int nfec_util_stream_copy(void* dst, const void* src, uint64_t bytes, void* stream);

/* ---- NORM wire format on the FEC path (host only; no device work) ----
 * The FEC Object Transmission Information header extension (type 64) a sender attaches to
 * NORM_INFO/NORM_DATA and a receiver reads to build its decoder, the FEC payload ID in every
 * NORM_DATA, and the codec choice each side makes from them.  Big-endian on the wire. */
typedef struct nfec_fti {
    uint8_t fec_id;         /* 2, 5 or 129 */
    uint8_t fec_m;          /* field bits: 8 or 16 for fec_id 2; 8 for 5 and 129 (read side) */
    uint8_t fec_group_size; /* fec_id 2 'G' (symbols per packet); read as 1 for 5, 129 */
    uint8_t reserved;
    uint16_t instance_id;   /* fec_id 129 */
    uint16_t segment_size;
    uint16_t num_data;      /* FEC max block length (u8 on the wire for fec_id 5) */
    uint16_t num_parity;
    uint64_t object_size;   /* NormObjectSize, 48 bits */
} nfec_fti;

/* NormFtiExtension2/5/129::SetObjectSize...SetFecNumParity (normMessage.h:785-1029):
 * writes the whole extension (16 bytes; 12 for fec_id 5) into ext and returns its length,
 * NFEC_EINVAL for an unknown fec_id, cap too small or object_size >= 2^48, NFEC_ERANGE when
 * num_data/num_parity do not fit fec_id 5's u8 fields. */
int nfec_fti_write(const nfec_fti* fti, void* ext, size_t cap);
/* The matching getters: parses ext (len bytes) for fec_id; returns bytes consumed or
 * NFEC_EINVAL (unknown fec_id, short buffer, type != 64 or length field too small). */
int nfec_fti_read(uint8_t fec_id, const void* ext, size_t len, nfec_fti* out);
/* NormPayloadId (normMessage.h:396-567): 4 bytes for fec_id 2 and 5, 8 for 129, 0 unknown. */
int nfec_payload_id_length(uint8_t fec_id);
/* fec 2/m 8 and fec 5: u32 block<<8 | symbol; fec 2/m 16: u16 block, u16 symbol; fec 129:
 * u32 block, u16 block length, u16 symbol.  Return the length, or NFEC_EINVAL.
 * block_len is only carried by fec 129 (read returns 0 for it otherwise; may be NULL). */
int nfec_payload_id_write(uint8_t fec_id, uint8_t fec_m, uint32_t block_id, uint16_t symbol_id,
                          uint16_t block_len, void* out);
int nfec_payload_id_read(uint8_t fec_id, uint8_t fec_m, const void* in, uint32_t* block_id,
                         uint16_t* symbol_id, uint16_t* block_len);
/* Sender choice (NormSession::StartSender, normSession.cpp:764-898): numParity == 0 -> no
 * codec (*kind = 0), fec_id_pref (0 = 5), m 8; numData + numParity <= 255 -> RS8 with
 * fec_id_pref (0 = 5) and m 8, or MDP/129 when assume_mdp; else RS16, fec 2, m 16. */
int nfec_sender_codec(uint16_t num_data, uint16_t num_parity, uint8_t fec_id_pref, int assume_mdp,
                      int* kind, uint8_t* fec_id, uint8_t* fec_m);
/* Receiver choice (NormSenderNode::AllocateBuffers, normNode.cpp:290-356): fec 2 m 8 -> RS8,
 * m 16 -> RS16; fec 5 -> RS8; fec 129 -> MDP when assume_mdp, RS8 for instance 0; anything
 * else NFEC_ENOTSUP. */
int nfec_receiver_codec(uint8_t fec_id, uint8_t fec_m, uint16_t instance_id, int assume_mdp,
                        int* kind);
/* The codec vector size for a segment size: segment_size + the 8-byte stream payload header
 * NORM codes along with the data (NormDataMsg::GetStreamPayloadHeaderLength). */
uint32_t nfec_vector_size(uint16_t segment_size);

/* ---- npc: the offline file precoder (src/common/normPrecode.cpp) on the GPU path ----
 * .npc files are byte-identical to the reference tool's for the same input and parameters
 * (meta segment, CRC-32 per segment, interleaving, the encoder's segment-id rotation). */
typedef struct nfec_npc_params {
    uint32_t segment_size;   /* "segment": 12..8192 bytes, the last 4 hold the segment's CRC-32 */
    uint32_t num_data;       /* "block": used when parity_fraction < 0 */
    uint32_t num_parity;     /* "parity" */
    double parity_fraction;  /* "auto" percent / 100; >= 0 sizes the block from the file size.
                                The reference's default is 100.0 (auto mode, 100x parity). */
    uint64_t b_max;          /* "bmax": auto-mode block cap */
    uint64_t i_max;          /* "imax": interleaver max dimension, 0 = none */
} nfec_npc_params;

typedef struct nfec_npc_layout {
    uint64_t num_segments;    /* segments in the .npc file */
    uint64_t input_segments;  /* meta + data segments */
    uint64_t num_blocks;
    uint32_t num_data, num_parity;
    uint32_t last_block_data;     /* numData of the last FEC block */
    uint32_t segment_size;
    uint32_t last_segment_bytes;  /* encode: file bytes in the last data segment (0 on decode) */
    int32_t kind;                 /* NFEC_RS8, or NFEC_RS16 when numData + numParity > 256 */
    uint64_t il_width, il_height, il_size, i_max;
} nfec_npc_layout;

/* NormPrecodeApp's constructor defaults (normPrecode.cpp:111-115). */
void nfec_npc_default_params(nfec_npc_params* params);
/* Block sizing (OnStartup :383-434) and file layout (Encode :611-637 / Decode :886-909,
 * InitInterleaver :450-462) for an input of file_size bytes.  Host only. */
int nfec_npc_layout_for(const nfec_npc_params* params, uint64_t file_size, int encode,
                        nfec_npc_layout* out);
/* File slot of FEC-order segments [first, first+count) (ComputeInterleaverOffset :465-556
 * divided by segment_size).  Host only.  NFEC_ENOTSUP where the reference's remap fails. */
int nfec_npc_positions(const nfec_npc_layout* layout, uint64_t first, uint64_t count, uint64_t* pos);
/* NormPrecodeApp::Encode: in_path -> out_path (.npc) on HIP device `device`. */
int nfec_npc_encode_file(int device, const char* in_path, const char* out_path,
                         const nfec_npc_params* params);
/* NormPrecodeApp::Decode: out_path NULL writes to the file name stored in the meta segment
 * (current directory), as the reference does; that name goes to name_out when given.
 * NFEC_ERANGE when a block has more bad segments than parity (the reference's fatal case). */
int nfec_npc_decode_file(int device, const char* in_path, const char* out_path,
                         const nfec_npc_params* params, uint64_t* out_bytes, char* name_out,
                         size_t name_cap);
/* The same file passes over several GPUs (devices[0..num_devices), may repeat a device):
 * device i takes the i-th contiguous range of FEC blocks, with its own codec, staging and host
 * thread; host copy threads (NFEC_NPC_THREADS) are shared among them.  Output bytes are
 * identical to the one-device call.  NFEC_EINVAL for an empty list or a device index out of
 * range.  The one-device functions above are these with a list of one. */
int nfec_npc_encode_file_multi(const int32_t* devices, int32_t num_devices, const char* in_path,
                               const char* out_path, const nfec_npc_params* params);
int nfec_npc_decode_file_multi(const int32_t* devices, int32_t num_devices, const char* in_path,
                               const char* out_path, const nfec_npc_params* params,
                               uint64_t* out_bytes, char* name_out, size_t name_cap);
/* CRC-32 (npc's ComputeCRC32, :1303-1313) of the first len bytes of slots [0, slots) of every
 * block of a device batch -> crc[b*slots + s] (device), asynchronously on stream. */
int nfec_crc32_slots(const nfec_block_batch* batch, uint32_t slots, uint32_t len, uint32_t* crc,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NFEC_H */

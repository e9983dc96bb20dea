/*
 * zd.h — C ABI of the MI355X-native ZSTD block-decode path.
 *
 * This is the drop-in boundary for the hot path of the reference crate
 * AchilleBailly/zstd-decompressor (Rust).  The reference has no FFI of its own;
 * its boundary is the public Rust API, and each entry point below names the
 * reference item it replaces (paths relative to the reference repo,
 * zstd-decompressor/src/…).  A Rust crate binds these with `extern "C"` blocks
 * (see INTEGRATION.md); the Python mirror in zstd-decompressor_amd/ binds them
 * with ctypes.
 *
 * Conventions
 *   - Every function returns ZD_OK (0) or a negative ZD_E_* code; nothing
 *     aborts across the ABI.
 *   - Plain pointers and sizes only.  `stream` parameters are hipStream_t
 *     passed as void* (NULL = default stream).
 *   - "d_" prefixed pointers are device (HBM) pointers, all others host.
 *   - The caller owns every buffer it passes; objects created by *_create /
 *     *_new own their own device memory and are released by *_destroy/_free.
 *   - Objects are not thread-safe; distinct objects may be used from
 *     distinct threads.
 */
#ifndef ZD_H
#define ZD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZD_ABI_VERSION 8

/* ------------------------------------------------------------------ */
/* Status codes: one per reference error variant (leaf of the          */
/* thiserror chain), plus codes for behaviour beyond the reference.    */
/* ------------------------------------------------------------------ */
#define ZD_OK 0
/* parsing::Error (parsing.rs:12-25) */
#define ZD_E_NOT_ENOUGH_BYTES              (-1)
#define ZD_E_NOT_ENOUGH_BITS               (-2)
#define ZD_E_MAX_READABLE_BITS_EXCEEDED    (-3)
#define ZD_E_EMPTY_INPUT_DATA              (-4)
#define ZD_E_NULL_BYTE                     (-5)
#define ZD_E_EMPTY_SLICE                   (-6)
/* decoders::Error (decoders/mod.rs:10-23) */
#define ZD_E_LARGE_ACCURACY_LOG            (-12)
#define ZD_E_CORRUPTED_TABLE               (-13)
#define ZD_E_SEQUENCE_CODE_MAX_EXCEEDED    (-14)
/* literals::Error (literals.rs:8-17) */
#define ZD_E_HUFFMAN_DECODER_MISSING       (-20)
#define ZD_E_CORRUPTED_STREAMS_SIZE        (-21)
/* sequences::Error (sequences.rs:14-23) */
#define ZD_E_SEQ_RESERVED_SET              (-30)
#define ZD_E_NO_PREVIOUS_DECODER           (-31)
/* decoding_context::Error (decoding_context.rs:8-15) */
#define ZD_E_CTX_WINDOW_SIZE_TOO_BIG       (-40)
#define ZD_E_NULL_OFFSET                   (-41)
#define ZD_E_IMPOSSIBLE_VALUE              (-42)
/* block::Error (block.rs:12-25) */
#define ZD_E_RESERVED_BLOCK_TYPE           (-50)
/* frame::Error (frame.rs:14-39) */
#define ZD_E_UNRECOGNIZED_MAGIC            (-60)
#define ZD_E_FRAME_RESERVED_SET            (-61)
#define ZD_E_MISSING_CHECKSUM              (-64)
#define ZD_E_WINDOW_SIZE_TOO_BIG           (-66)
/* Beyond the reference */
#define ZD_E_REF_PANIC       (-90) /* the reference would panic / not terminate here */
#define ZD_E_OUT_OF_DOMAIN   (-91) /* input outside the GPU path's parity domain */
#define ZD_E_DST_TOO_SMALL   (-92)
#define ZD_E_INVALID_ARG     (-93)
#define ZD_E_HIP             (-94) /* a HIP runtime call failed */
#define ZD_E_NO_MEMORY       (-95)
#define ZD_E_NOT_DECODED     (-96) /* frame skipped: an earlier frame failed (FrameIterator stops, frame.rs:94-99) */
#define ZD_E_COMM            (-97) /* an RCCL call failed, or RCCL is not loadable */

/* Device workspaces of destroyed plans are kept for reuse by later plans of
 * the process (bounded by ZD_WS_CACHE_MB, default 8 GiB; 0 disables it).
 * zd_trim_cache frees them (every device): PyTorch's caching allocator does
 * not see this memory. */
void zd_trim_cache(void);

/* Human-readable name of a status code (static storage). */
const char* zd_status_name(int status);
int zd_abi_version(void);

/* ------------------------------------------------------------------ */
/* Frame index — replaces FrameIterator::next + Frame::parse +        */
/* Header::parse + Block::parse (frame.rs:61-99,111-177,198-230;       */
/* block.rs:43-72).  Host-side, O(frames+blocks), reads only headers.  */
/* ------------------------------------------------------------------ */
#define ZD_FRAME_ZSTD      0
#define ZD_FRAME_SKIPPABLE 1

typedef struct zd_frame_desc {
  uint64_t src_offset;     /* offset of the 4-byte magic in src */
  uint64_t src_size;       /* bytes of the whole frame (header, blocks, checksum) */
  uint64_t content_size;   /* Frame_Content_Size, UINT64_MAX if absent */
  uint64_t window_size;    /* Header::window_size (frame.rs:105) */
  uint64_t dict_id;        /* Header::dictionnary_id, UINT64_MAX if absent */
  uint32_t magic;
  uint32_t kind;           /* ZD_FRAME_ZSTD / ZD_FRAME_SKIPPABLE */
  uint32_t first_block;    /* index into the block array */
  uint32_t num_blocks;
  uint32_t has_checksum;
  uint32_t checksum;       /* ZStandard::checksum() (frame.rs:268) */
} zd_frame_desc;

#define ZD_BLOCK_RAW        0
#define ZD_BLOCK_RLE        1
#define ZD_BLOCK_COMPRESSED 2

typedef struct zd_block_desc {
  uint64_t src_offset;     /* first byte after the 3-byte block header */
  uint32_t block_size;     /* Block_Size field (block.rs:50) */
  uint8_t  type;           /* ZD_BLOCK_* */
  uint8_t  last;
  uint8_t  rle_byte;       /* RLEBlock::byte */
  uint8_t  _pad;
} zd_block_desc;

/*
 * Walk the frames of src[0..n).  With frames == NULL (or cap_frames == 0) the
 * whole input is walked and *nframes / *nblocks receive the totals (size
 * query); otherwise at most cap_frames frames are indexed, and blocks beyond
 * cap_blocks are counted but not stored.  *consumed = bytes of the indexed
 * frames (Frame::parse advances the parser the same way).  Stops at the first frame that fails
 * to parse, like FrameIterator + the CLI loop (src/main.rs:43-53): the
 * return value is that frame's status and *consumed the byte offset of the
 * failing frame (n on full success).  Table-level parse errors (FSE/Huffman
 * descriptions) are found on the GPU, not here.
 */
int zd_frames_index(const uint8_t* src, size_t n,
                    zd_frame_desc* frames, size_t cap_frames, size_t* nframes,
                    zd_block_desc* blocks, size_t cap_blocks, size_t* nblocks,
                    size_t* consumed);

/* ------------------------------------------------------------------ */
/* Batch decode (the hot path): a plan over a byte range of frames.    */
/* Replaces Frame::decode / ZStandard::decode (frame.rs:79-84,232-260) */
/* and, per block, Block::decode (block.rs:74-99) with HIP kernels.    */
/* ------------------------------------------------------------------ */
typedef struct zd_plan zd_plan;

#define ZD_F_SKIPPABLE  1u  /* append skippable-frame payloads to the output (CLI -p, src/main.rs:45-48) */
/* Executor choice for frames of many blocks; default:
 * automatic.  Same output either way; tests run both. */
#define ZD_F_BLOCK_PARALLEL 2u  /* every frame with a compressed block -> K4J (block-parallel execute) */
#define ZD_F_FRAME_SERIAL   4u  /* no frame -> K4J (the streaming per-frame executor) */
/* Sequence-decode choice: K3 with one lane per block instead of four (the
 * default, K3Q).  Same records either way; tests run both. */
#define ZD_F_SEQ_ONE_LANE   8u
/* Launch choice for plans of 256-1024 single-block frames:
 * K3 and K4 run fused per frame group (zd_k_fused) by default; this flag
 * keeps them as two launches.  Same output either way; tests run both. */
#define ZD_F_NO_FUSE      32u
/* Table-build choice for plans of up to 16,384 tables: K1's sequence half
 * runs one wave per block by default; this flag keeps K1's serial lanes.
 * Same tables either way; tests run both. */
#define ZD_F_K1_LANES     64u
/* Sequence-decode choice for plans of few blocks (<= 8 per CU): K3 runs
 * one block per wave (zd_k_sequences_l, latency-first) by default; this flag
 * keeps K3Q.  Same records either way; tests run both. */
#define ZD_F_SEQ_NO_LATENCY 256u
/* Test switch: K4J runs ONE pointer-jumping round of one hop, so a frame
 * whose match chains are deeper keys LS_JROUNDS and zd_plan_decompress plans
 * it again on the streaming executor (tests/test_large_frames.py). */
#define ZD_F_J_ONE_ROUND 128u

/* zd_plan_info.executors: */
#define ZD_EXEC_FUSED 1u   /* zd_k_fused: tables, FSE chains and execution per group of four
                              single-block frames (not while kernel profiling is on) */
#define ZD_EXEC_K4F   2u   /* some frames execute resident in LDS (zd_k_execute_lds) */
#define ZD_EXEC_K4J   4u   /* some frames execute block-parallel (pointer jumping) */

typedef struct zd_plan_info {
  uint64_t nframes;        /* frames in the plan (skippable included) */
  uint64_t nblocks;
  uint64_t ncompressed;    /* compressed blocks */
  uint64_t src_bytes;      /* bytes of src covered by the plan */
  uint64_t out_bytes;      /* exact decoded size if every frame has a FCS, else an upper bound */
  uint64_t out_exact;      /* 1 if out_bytes is exact */
  uint64_t workspace_bytes;/* device workspace owned by the plan */
  uint64_t nsequences;     /* sum of Number_of_Sequences over compressed blocks */
  uint64_t nliterals;      /* sum of Regenerated_Size over compressed-literal blocks */
  int32_t  index_status;   /* status of the host walk (first failing frame) */
  uint32_t executors;      /* ZD_EXEC_* bits: the executors the plan's frames take */
  uint64_t host_ns;        /* zd_plan_create: header walk + descriptors (host work) */
  uint64_t device_ns;      /* zd_plan_create: workspace allocation + descriptor upload */
  uint64_t walk_serial_bytes; /* input bytes the frame walk had to walk serially (a range whose
                                 parallel walk started at a magic number inside data); 0 normally */
  uint64_t io_h2d_ns;      /* the last zd_plan_decompress: input host -> HBM */
  uint64_t io_decode_ns;   /*   decode + results (kernels, status read-back) */
  uint64_t io_d2h_ns;      /*   output HBM -> host */
  uint64_t error_key;      /* the last zd_plan_results: where the first failing frame stopped,
                              phase << 62 | block in frame << 32 | stage << 28 | sub << 8 | -status
                              (phase 0 parse, 1 decode, 3 a limit of the GPU path; stages
                              csrc/zd_common.h); all ones when every frame decoded */
  uint64_t replans;        /* the last zd_plan_decompress: re-plans past frames that overran
                              their reserved capacity (or K4J rounds), 0 normally */
  uint64_t fused_redo_frames; /* the last zd_plan_results of a zd_k_fused launch: frames its redo
                              pass decoded (a fast-chain reject, or a wait for K2 / the chain
                              past its bound); 0 normally, never a different output */
  uint64_t device_descriptors; /* 1: zd_plan_create_device built the descriptors on the GPU from its
                              own index (only the frames' output offsets and capacities came
                              back); 0: the index came back and the host built them */
} zd_plan_info;

/* The executor routing zd_plan_create / zd_decode_async choose for a plan of
 * this shape on a device of `cus` compute units (host only: diagnostics and
 * tests).  Every bound scales with the CU count (zd_host.cpp route_plan,
 * DESIGN.md §4): single_block_frames = every frame one compressed block.
 * *route = ZD_ROUTE_* bits. */
#define ZD_ROUTE_FUSED        1u   /* zd_k_fused (tables + K3 + K4 per group of four frames) */
#define ZD_ROUTE_K4F          2u   /* frames up to 128 KiB execute resident in LDS */
#define ZD_ROUTE_K1_SEQ_WAVES 4u   /* K1's sequence half one wave per block */
#define ZD_ROUTE_FORK         8u   /* K2 beside K3 on a second stream */
#define ZD_ROUTE_K1_FORK     16u   /* K1's two halves on the two streams */
int zd_route(uint32_t cus, uint64_t nframes, uint64_t n_tables, uint64_t n_seq_blocks, uint64_t n_huf_blocks,
             int single_block_frames, uint32_t flags, uint32_t* route);

/* Index src[0..n) on the host and allocate the plan's device workspace.
 * Host-side work only (no kernel launches).  A frame that fails to index
 * ends the plan (its status is kept and reported by zd_plan_results). */
int zd_plan_create(const uint8_t* src, size_t n, uint32_t flags, zd_plan** out);
/* The same plan from an input resident in device memory only (d_src,
 * readable for n + ZD_SRC_PADDING bytes): the frame / block header walk runs
 * on the GPU (zd_k_walk, one wave per byte range, the host walk's own code in
 * zd_walk.h), and only its index -- frames and blocks, about 150 bytes per
 * block -- comes back to the host for the descriptors.  Replaces the host
 * pre-pass of FrameIterator / Frame::parse / Header::parse / Block::parse
 * and the section headers (frame.rs:61-230, block.rs:43-72,
 * literals.rs:88-206, sequences.rs:52-143) for input that never was in host
 * memory (e.g. a frame range received from another GPU).  The plan equals
 * zd_plan_create's on the same bytes.  Synchronises `stream`. */
int zd_plan_create_device(const uint8_t* d_src, size_t n, uint32_t flags, void* stream, zd_plan** out);
int zd_plan_info_get(const zd_plan* plan, zd_plan_info* info);
/* Waits for the work the plan launched, then returns its device workspace to
 * the process cache (zd_trim_cache). */
void zd_plan_destroy(zd_plan* plan);

/* Bitstream readers fetch aligned 16-byte windows and may touch up to
 * ZD_SRC_PADDING bytes past the end of the input: device input buffers must
 * stay readable that far (the contents there do not matter). */
#define ZD_SRC_PADDING 16

/* Launch the decode pipeline on `stream`.  d_src holds the same n bytes
 * given to zd_plan_create, resident in HBM (readable for n + ZD_SRC_PADDING
 * bytes); d_dst receives the
 * concatenated output (>= info.out_bytes).  No host synchronisation, no
 * allocation: safe to capture in a hipGraph. */
int zd_decode_async(zd_plan* plan, const uint8_t* d_src, uint8_t* d_dst,
                    size_t dst_cap, void* stream);

/* After the stream has drained: per-frame status and decoded length
 * (host arrays of plan nframes entries, either may be NULL), the total
 * length of the CLI-style output (frames up to the first failure) and the
 * overall status (first failing frame's status, or ZD_OK).  If some frame
 * had no FCS this also compacts d_dst in place so the frames are
 * contiguous (needs the same d_dst and stream). */
int zd_plan_results(zd_plan* plan, uint8_t* d_dst, void* stream,
                    int32_t* frame_status, uint64_t* frame_len,
                    uint64_t* total_len, int32_t* first_error_frame);

/* Content checksums, an extra beyond the reference: after zd_plan_results
 * (same d_dst and stream), XXH64 (seed 0) of every decoded frame's output,
 * computed on the GPU.  ok[i] = 1 when frame i carries a Content_Checksum and
 * it equals the digest's low 32 bits, 0 when it differs, -1 when the frame has
 * none or was not decoded; hash[i] = the digest (0 if not decoded).  The
 * reference computes the hash but never enforces it (frame.rs:239-255,
 * SURVEY D5), so a mismatch never changes the decode status.  Host arrays of
 * plan nframes entries, either may be NULL. */
int zd_plan_checksums(zd_plan* plan, const uint8_t* d_dst, void* stream, int32_t* ok, uint64_t* hash);

/* Kernel times of the last zd_decode_async on the plan, in ms (HIP events on
 * the plan's stream).  zd_plan_set_profiling mode 1: every kernel timed, the
 * launches one after another (no K2 | K3 fork, no fused kernel); mode 2: the
 * pipeline exactly as it runs unprofiled, with events around each launch
 * group that can carry the plan's work and did launch, one entry each, in
 * this order: "zd_k_rawcopy" (K0, raw/RLE blocks), "zd_k_fused", "zd_k_execute"
 * (only when some frame runs on it), "zd_k_execute_lds" (K4F), and the K4J
 * kernels together ("zd_k_jsum+...+zd_k_jround"); the largest is the
 * dominant launch.  0: off.  names/ms arrays of cap entries. */
int zd_plan_set_profiling(zd_plan* plan, int enable);
int zd_plan_kernel_times(zd_plan* plan, const char** names, float* ms, int cap, int* n);

/* zd_decompress with a plan already made for the same n bytes (so a caller
 * that sized dst from zd_plan_info_get does not plan twice).  The plan keeps
 * the device buffers for the next call (freed by zd_plan_destroy); input and
 * output move through pinned chunks (zd_plan_info io_*_ns: the phases of the
 * last call).  A frame that decodes past the capacity the plan reserved for
 * it (its Frame_Content_Size, or 128 KiB per block) is planned again from its
 * own start with more room, as often as needed (info.replans); the reference
 * checks neither (decoding_context.rs:29-47, block.rs:50).  Calls on distinct
 * plans may run on distinct threads (thread safe: they share one
 * process-wide pair of pinned chunks only while copying).  Every call runs on
 * the device's legacy null stream, so concurrent calls do not overlap on the
 * GPU; a caller that wants overlap uses zd_decode_async on its own streams.
 * One plan is not used from two threads at once. */
int zd_plan_decompress(zd_plan* plan, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);
/* Per-frame outcome of the last zd_plan_decompress on the plan (its re-plans
 * included): frame f's status (ZD_OK, the frame's error, or
 * ZD_E_NOT_DECODED after the first failing frame) and where its bytes sit in
 * dst (offset, length; length 0 unless ZD_OK).  *n = the plan's frames
 * (0 before any call); arrays of cap entries, any may be NULL.  This is what
 * a FrameIterator-style caller (frame.rs:86-99) hands out frame by frame
 * from one decode of the whole buffer. */
int zd_plan_frame_outputs(const zd_plan* plan, int32_t* status, uint64_t* offset, uint64_t* length, size_t cap,
                          size_t* n);
/* Convenience: host in, host out (H2D + decode + D2H on the default
 * stream).  Mirrors the CLI (src/main.rs:43-58) minus the UTF-8 step. */
int zd_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                  size_t* out_len, uint32_t flags);

/* ------------------------------------------------------------------ */
/* Multi-GPU: frame-range sharding + RCCL gather.      */
/* Frames are independent (a fresh DecodingContext each, frame.rs:     */
/* 232-237) and the CLI concatenates their outputs, stopping at the    */
/* first failing frame (src/main.rs:43-53).  One process per GPU; each */
/* rank decodes a contiguous frame range into its own HBM (no data-    */
/* path collective), then the ranges are gathered to rank 0.           */
/* ------------------------------------------------------------------ */

/* Contiguous frame ranges balanced by compressed bytes: rank k takes
 * frames [cuts[k], cuts[k+1]) (cuts has world + 1 entries; every rank gets a
 * frame while there are at least `world`).  Host only. */
int zd_shard_partition(const uint64_t* frame_bytes, size_t nframes, int world, size_t* cuts);

/* Rank's share of src: byte range [*src_begin, *src_end) and frame range
 * (frames indexed on the host with zd_frames_index).  A frame that fails
 * to index and the rest of the input go to the last rank, whose plan then
 * reports it.  Host only. */
int zd_shard_range(const uint8_t* src, size_t n, int rank, int world, uint64_t* src_begin, uint64_t* src_end,
                   uint64_t* frame_begin, uint64_t* frame_end);

/* Every rank's share at once, from one walk of the input: rank k's bytes are
 * [src_cuts[k], src_cuts[k+1]) and its frames [frame_cuts[k],
 * frame_cuts[k+1]) (world + 1 entries each), exactly zd_shard_range's.  Made
 * once (on one rank, or ahead of time and kept beside the input) and handed
 * to the ranks, so that no rank walks frames outside its own range.  Host
 * only. */
int zd_shard_cuts(const uint8_t* src, size_t n, int world, uint64_t* src_cuts, uint64_t* frame_cuts);

/* zd_shard_range from given cuts, in time O(the rank's own range): walks only
 * the rank's frames and checks that they tile its byte range with its frame
 * count (the last rank's range may end in a frame that fails to index).
 * ZD_E_INVALID_ARG when they do not, i.e. the cuts are not this input's.
 * Host only. */
int zd_shard_range_at(const uint8_t* src, size_t n, const uint64_t* src_cuts, const uint64_t* frame_cuts, int rank,
                      int world, uint64_t* src_begin, uint64_t* src_end, uint64_t* frame_begin,
                      uint64_t* frame_end);

typedef struct zd_comm zd_comm;
#define ZD_COMM_ID_BYTES 128

/* An RCCL communicator over `world` ranks, one GPU each (the calling
 * thread's current HIP device).  Rank 0 makes the id and shares it out of
 * band (e.g. a torch.distributed broadcast); every rank then calls
 * zd_comm_create with it.  RCCL is loaded on first use. */
int zd_comm_unique_id(uint8_t id[ZD_COMM_ID_BYTES]);
int zd_comm_create(const uint8_t id[ZD_COMM_ID_BYTES], int world, int rank, zd_comm** out);
void zd_comm_destroy(zd_comm* comm);
/* The device buffers zd_decode_sharded keeps in the communicator between
 * calls (its input copy and its own output buffer), in bytes: memory
 * accounting.  A rank-0 decode that outgrows the caller's d_root_out moves to
 * an output buffer sized from what it needs, never from root_cap. */
int zd_comm_buffers(const zd_comm* comm, uint64_t* src_bytes, uint64_t* out_bytes);

typedef struct zd_gather_result {
  uint64_t total_len;         /* bytes gathered on rank 0 */
  int32_t status;             /* the whole input's status: the first failing rank's */
  int32_t failed_rank;        /* that rank, or world when none failed */
  int64_t first_error_frame;  /* global index of the first failing frame, -1 if none */
} zd_gather_result;

/* Host only: the outcome merge every rank of zd_comm_gather performs on the
 * all-gathered outcomes.  meta = world x 4 int64 {status, first failing frame
 * (global, -1 if none), local length, root capacity (rank 0's entry; 0
 * elsewhere)}.  The output stops at the first failing rank's failure: that
 * rank keeps its frames before the failure (its local length), later ranks
 * contribute nothing (src/main.rs:43-53).  Fills off[r] / len[r] (world
 * entries: where rank r's bytes land on rank 0, and how many) and *res;
 * returns ZD_E_DST_TOO_SMALL (res->total_len 0: nothing may be sent) when the
 * kept bytes exceed rank 0's capacity. */
int zd_gather_layout(const int64_t* meta, int world, uint64_t* off, uint64_t* len, zd_gather_result* res);

/* Collective (every rank calls it): each rank's outcome — status, first
 * failing frame (global index), decoded length — is all-gathered; the output
 * stops at the first failing rank's failure (its frames before the failure
 * kept, later ranks contribute nothing), and rank 0 receives the ranks'
 * d_local bytes in rank order at d_root_out (capacity root_cap; rank 0's own
 * bytes are copied unless d_local == d_root_out) with RCCL point-to-point
 * transfers on `stream`.  The same *res on every rank.  ZD_E_DST_TOO_SMALL
 * (on every rank, nothing sent) when rank 0's capacity is short. */
int zd_comm_gather(zd_comm* comm, const uint8_t* d_local, uint64_t local_len, int32_t status,
                   int64_t first_error_frame, uint8_t* d_root_out, uint64_t root_cap, zd_gather_result* res,
                   void* stream);

/* The whole multi-GPU decode (the reference's `decode every frame of a
 * file`, sharded): every rank passes the same host input; rank `comm`'s
 * frame range is planned, copied to HBM, decoded (with zd_plan_decompress's
 * re-plans past frames that overran their reserved capacity), and gathered
 * to rank 0 (zd_comm_gather).  Returns the local call's status (ZD_OK when
 * the collective completed); the input's status is res->status. */
int zd_decode_sharded(zd_comm* comm, const uint8_t* src, size_t n, uint32_t flags, uint8_t* d_root_out,
                      uint64_t root_cap, zd_gather_result* res, void* stream);

/* zd_decode_sharded with the ranks' cuts given (zd_shard_cuts): each rank
 * walks and plans only its own range.  A rank whose range does not fit the
 * cuts still joins the collective: res->status is then ZD_E_INVALID_ARG on
 * every rank. */
int zd_decode_sharded_at(zd_comm* comm, const uint8_t* src, size_t n, const uint64_t* src_cuts,
                         const uint64_t* frame_cuts, uint32_t flags, uint8_t* d_root_out, uint64_t root_cap,
                         zd_gather_result* res, void* stream);

/* ------------------------------------------------------------------ */
/* DecodingContext mirror (decoding_context.rs:17-106): GPU-resident    */
/* per-frame state across Block::decode calls.                         */
/* ------------------------------------------------------------------ */
typedef struct zd_context zd_context;

/* DecodingContext::new (decoding_context.rs:29-47): fails with
 * ZD_E_CTX_WINDOW_SIZE_TOO_BIG above 8 MiB. */
int zd_context_new(uint64_t window_size, zd_context** out);
void zd_context_free(zd_context* ctx);

/* Block::parse + Block::decode (block.rs:43-99) on the GPU: parses one
 * block (3-byte header + content) from src[0..n), decodes it on the
 * device appending to the context.  *consumed / *last as Block::parse. */
int zd_block_decode(zd_context* ctx, const uint8_t* src, size_t n,
                    size_t* consumed, int* last);

/* DecodingContext::execute_sequences (decoding_context.rs:78-106) on the
 * GPU: sequences are (literals_length, offset_value, match_length), any u32
 * values.  ZD_E_OUT_OF_DOMAIN when the context's output would pass
 * 2^31 - 64 KiB (the streaming executor's positions). */
int zd_execute_sequences(zd_context* ctx, const uint32_t* ll,
                         const uint32_t* offset_value, const uint32_t* ml,
                         size_t nseq, const uint8_t* literals, size_t nlits);

/* DecodingContext::decoded / ::offsets (decoding_context.rs:19-20). */
int zd_context_decoded(const zd_context* ctx, uint8_t* dst, size_t cap, size_t* len);
int zd_context_offsets(const zd_context* ctx, uint64_t offsets[3]);

#ifdef __cplusplus
}
#endif
#endif /* ZD_H */

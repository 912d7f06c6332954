/*
 * wsframe_amd.h — C ABI of the MI355X WebSocket frame-decode engine
 * (libwsframe_amd.so). Drop-in for hujianzhe/util crt/protocol/websocketframe.
 *
 * Part 1 re-exports the eight reference symbols with identical signatures and
 * semantics (inc/crt/protocol/websocketframe.h:42-49). They work on host
 * memory, one frame / one handshake at a time, exactly like the reference, so
 * existing callers (user glue behind NetChannelExProc_t.on_decode,
 * inc/component/net_channel_ex.h:22-27) link unchanged.
 *
 * Part 2 is the batch API the GPU path adds: a device-resident
 * batch of rx segments (one per connection inbuf, src/component/net_reactor.c
 * :465-545) is decoded by hand-written gfx950 kernels with the exact semantics
 * of the reactor's per-frame loop (net_reactor.c:515-526) running
 * websocketframeDecode (websocketframe.c:112-165) on every segment.
 *
 * Plain pointers and sizes only; no torch types. Every pointer named d_* is
 * device memory, h_* is host memory. Buffers are owned by the caller; the
 * library never frees user memory.
 */
#ifndef UTIL_AMD_WSFRAME_AMD_H
#define UTIL_AMD_WSFRAME_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define WSFRAME_AMD_EXPORT __attribute__((visibility("default")))

/* ---- Part 1: reference ABI (websocketframe.h:10-19, :42-49) ---------------- */

enum {
    WEBSOCKET_CONTINUE_FRAME = 0,
    WEBSOCKET_TEXT_FRAME = 1,
    WEBSOCKET_BINARY_FRAME = 2,
    WEBSOCKET_CLOSE_FRAME = 8,
    WEBSOCKET_PING_FRAME = 9,
    WEBSOCKET_PONG_FRAME = 10
};

#define WEBSOCKET_MAX_ENCODE_HEADLENGTH 10

/* websocketframe.h:21-36: the client handshake request templates (path, key[, protocol]) */
#define WEBSOCKET_SIMPLE_HTTP_HANDSHAKE_REQUEST_FMT \
    "GET %s HTTP/1.1\r\n"                          \
    "Upgrade: websocket\r\n"                       \
    "Connection: Upgrade\r\n"                      \
    "Sec-WebSocket-Version: 13\r\n"                \
    "Sec-WebSocket-Key: %s\r\n"                    \
    "\r\n"

#define WEBSOCKET_SIMPLE_HTTP_HANDSHAKE_REQUEST_WITH_PROTOCOL_FMT \
    "GET %s HTTP/1.1\r\n"                                        \
    "Upgrade: websocket\r\n"                                     \
    "Connection: Upgrade\r\n"                                    \
    "Sec-WebSocket-Version: 13\r\n"                              \
    "Sec-WebSocket-Key: %s\r\n"                                  \
    "Sec-WebSocket-Protocol: %s\r\n"                             \
    "\r\n"

/* websocketframe.c:16-32 */
WSFRAME_AMD_EXPORT char* websocketframeComputeSecAccept(const char* sec_key, unsigned int sec_keylen,
                                                        char sec_accept[60]);
/* websocketframe.c:34-73 */
WSFRAME_AMD_EXPORT int websocketframeDecodeHandshakeRequest(const char* data, unsigned int datalen,
                                                            const char** sec_key, unsigned int* sec_keylen,
                                                            const char** sec_protocol,
                                                            unsigned int* sec_protocol_len);
/* websocketframe.c:75-84 */
WSFRAME_AMD_EXPORT char* websocketframeEncodeHandshakeResponse(const char* sec_accept,
                                                               unsigned int sec_accept_len, char buf[162]);
/* websocketframe.c:86-108 */
WSFRAME_AMD_EXPORT char* websocketframeEncodeHandshakeResponseWithProtocol(const char* sec_accept_key,
                                                                           unsigned int sec_accept_len,
                                                                           const char* sec_protocol,
                                                                           unsigned int sec_protocol_len);
/* websocketframe.c:110 */
WSFRAME_AMD_EXPORT void websocketframeFreeString(char* s);
/* websocketframe.c:112-165 */
WSFRAME_AMD_EXPORT int websocketframeDecode(unsigned char* buf, unsigned long long len, unsigned char** data,
                                            unsigned long long* datalen, int* is_fin, int* type);
/* websocketframe.c:167-174 */
WSFRAME_AMD_EXPORT unsigned int websocketframeEncodeHeadLength(unsigned long long datalen);
/* websocketframe.c:176-202 */
WSFRAME_AMD_EXPORT void websocketframeEncode(void* headbuf, int is_fin, int prev_is_fin, int type,
                                             unsigned long long datalen);

/* ---- Part 2: batch decode on MI355X ------------------------------------------ */

/* Per-frame result: the four out-params of websocketframeDecode plus its
 * return value and the frame's position. 32 bytes, naturally aligned. */
typedef struct WebsocketFrameDesc_t {
    unsigned long long frame_off; /* wire offset of the frame from the batch buffer base */
    unsigned long long data_off;  /* payload offset from the buffer base; ~0ULL where *data == NULL */
    unsigned long long datalen;   /* *datalen */
    int ret;                      /* websocketframeDecode return value (never 0 in a descriptor) */
    unsigned char is_fin;         /* *is_fin */
    unsigned char type;           /* *type (raw 4-bit opcode, not validated, as the reference) */
    unsigned char masked;         /* MASK bit of byte 1 */
    unsigned char hdrlen;         /* 2 + ext + mask bytes */
} WebsocketFrameDesc_t;

#define WEBSOCKET_DATA_OFF_NULL (~0ULL)

/* Segment stop reasons (WebsocketSegResult_t.status) */
enum {
    WEBSOCKET_SEG_OK = 0,              /* consumed everything, or stopped at an incomplete tail (ret 0) */
    WEBSOCKET_SEG_MAX_FRAMES = 1,      /* descriptor capacity reached; resubmit from `consumed` */
    WEBSOCKET_SEG_ERR_DECODE = -1,     /* a frame returned ret < 0 (int truncation, websocketframe.c:164):
                                          the reactor marks the channel invalid (net_reactor.c:518-520) */
    WEBSOCKET_SEG_ERR_LEN_WRAP = -2,   /* masked frame whose u64 length sum wraps (websocketframe.c:149):
                                          the reference would unmask past the buffer (undefined behaviour);
                                          fenced off here, nothing is written for that frame */
    WEBSOCKET_SEG_ERR_OUT_SPACE = -3,  /* reassembly only: the bodies outgrow the segment's output region
                                          (possible only through the (int) return truncation of frames
                                          >= 2 GiB, websocketframe.c:164) */
    WEBSOCKET_SEG_ERR_CACHE_OVERFLOW = -4 /* reassembly only: caching this frame's body would take the
                                          connection's cached bytes past readcache_max_size
                                          (check_cache_overflow, net_channel_ex.c:45-53,132-135); the
                                          reactor detaches the channel (NET_REACTOR_CACHE_READ_OVERFLOW_ERR).
                                          Its descriptor is written and counted in n_frames, it is not
                                          consumed, and no body or message is emitted for it */
};

/* Per-segment result. 16 bytes. */
typedef struct WebsocketSegResult_t {
    unsigned long long consumed; /* Σ ret of decoded frames = bytes the reactor would drop from inbuf */
    unsigned int n_frames;       /* descriptors written for this segment */
    int status;                  /* WEBSOCKET_SEG_* */
} WebsocketSegResult_t;

/* Device batches must keep WEBSOCKET_BATCH_PAD readable bytes of device memory
 * after the end of every segment (e.g. allocate the highest segment end + 32).
 * The kernels may read those bytes (never write them, never use their values):
 * it lets every header fetch be one unconditional scalar load. */
#define WEBSOCKET_BATCH_PAD 32

/* Decode a device-resident batch of rx segments in place, asynchronously on
 * `hip_stream` (hipStream_t, NULL = default stream).
 *   d_buf          batch buffer (device); payloads are unmasked in place
 *   buflen         every segment lies in [0, buflen) of d_buf; d_buf[0, buflen + WEBSOCKET_BATCH_PAD)
 *                  must be readable (the kernels read, never write, bytes outside segments;
 *                  bytes inside a segment that the decode does not change may be written
 *                  back with their own value — whole 16-B stores)
 *   d_seg_off/len  nseg segments [off, off+len) of d_buf (device arrays); must not overlap;
 *                  ascending order is fastest (any order is decoded correctly)
 *   max_frames     descriptor capacity per segment (>= 1)
 *   d_desc_base    optional (device, may be NULL): first descriptor slot of segment s;
 *                  NULL means s * max_frames
 *   d_desc         descriptor array (device)
 *   d_res          nseg segment results (device)
 * Semantics: for every segment, bit-identical to running
 *   off = 0; while (off < len) { r = websocketframeDecode(buf+off, len-off, ...);
 *                                if (r < 0) error; if (r == 0) break; off += r; }
 * (net_reactor.c:515-526), including every reference quirk (§SURVEY 4).
 * Concurrency: every HIP stream (up to 16 per device) gets its own workspace, so calls
 * on different streams — several rx batches in flight, one stream each, from one or
 * several host threads — may overlap in time (batches must not share bytes). The first
 * call on a stream (and a call on a larger batch) may allocate: make it before capturing
 * calls into a HIP graph.
 * Returns 0, or a negative code if the launch failed (see websocketframeGpuLastError). */
WSFRAME_AMD_EXPORT int websocketframeBatchDecodeDevice(unsigned char* d_buf, unsigned long long buflen,
                                                       const unsigned long long* d_seg_off,
                                                       const unsigned long long* d_seg_len, unsigned int nseg,
                                                       unsigned int max_frames,
                                                       const unsigned long long* d_desc_base,
                                                       WebsocketFrameDesc_t* d_desc, WebsocketSegResult_t* d_res,
                                                       void* hip_stream);

/* Same, but buffers live in host memory (the reactor's m_inbuf), synchronous.
 * Segment offsets are relative to h_buf. Pipelined: groups of consecutive
 * ascending segments (~64 MiB, option "host_chunk_mb") are copied H2D, decoded
 * and copied back D2H on three streams, so both copy directions and the kernel
 * overlap; any other segment layout is one group. Only segment bytes are written
 * back to h_buf (bytes between segments are read, never written). Pass pinned memory
 * (hipHostMalloc / hipHostRegister) for asynchronous DMA; pageable memory works
 * through the runtime's staging copies. h_desc must hold nseg*max_frames
 * descriptors (desc_base form not offered); slots past n_frames are zeroed. The
 * calling thread's current HIP device is unchanged on return. */
WSFRAME_AMD_EXPORT int websocketframeBatchDecodeHost(unsigned char* h_buf, unsigned long long buflen,
                                                     const unsigned long long* h_seg_off,
                                                     const unsigned long long* h_seg_len, unsigned int nseg,
                                                     unsigned int max_frames, WebsocketFrameDesc_t* h_desc,
                                                     WebsocketSegResult_t* h_res, int device);

/* The same on several devices (one host rx arena, every device's PCIe link carrying a share;
 * net_reactor.c:484-500 keeps every connection's m_inbuf in host memory): ascending,
 * non-overlapping segments are cut into ndev contiguous ranges of about equal bytes (at the
 * segment boundary nearest to each equal share) and each range runs
 * websocketframeBatchDecodeHost's pipeline on devices[i] from its own host thread; results land
 * in h_desc / h_res exactly where the one-device call puts them. A device may be listed more than
 * once (its ranges then run one after the other). Any other segment layout (unordered,
 * overlapping) or ndev == 1 is the one-device call on devices[0]. Synchronous; returns 0 or the
 * first failing range's error (websocketframeGpuLastError names its device). */
WSFRAME_AMD_EXPORT int websocketframeBatchDecodeHostMulti(unsigned char* h_buf, unsigned long long buflen,
                                                          const unsigned long long* h_seg_off,
                                                          const unsigned long long* h_seg_len, unsigned int nseg,
                                                          unsigned int max_frames, WebsocketFrameDesc_t* h_desc,
                                                          WebsocketSegResult_t* h_res, const int* devices, int ndev);

/* One raw rx stream of any size (a single connection's inbuf; no frame offsets from the
 * host): identical results to websocketframeBatchDecodeDevice with the one segment
 * [0, len) (descriptors d_desc[0..], result d_res[0]); WEBSOCKET_BATCH_PAD readable bytes
 * after d_buf + len. Frame boundaries are found by grid-wide speculative passes (one
 * probe + rest pair per change of frame length); the loop's state stays on the device (the
 * last block of each pass applies its stop), so the call is asynchronous and may be
 * captured in a HIP graph: "stream_rounds" pass pairs (default 4), then, on a stream of
 * >= 512 KiB, the chunk-parallel walk below with its geometry chosen and its chunk records
 * linked on the device (scratch sized from len when captured: about 2-5 % of len), on a
 * shorter one a single wavefront. An eager call on a stream of >= 512 KiB waits for the state
 * each round publishes to pinned host memory (no copy): more rounds while they pay, and once
 * lengths keep changing (>= 512 KiB and >= 256 frames left) the chunk-parallel walk
 * (speculative chunk entries, chunks of ~1024 mean frames up to 4 MiB by default, each written
 * by one wavefront). While the previous chunk walk on the same stream (or the previous replay of
 * a captured call) saw lengths that keep changing, the pass rounds are skipped and the walk
 * starts at 0: results never depend on this. Workspace and scratch are per
 * (stream, graph capture), so calls on different streams may overlap. Returns 0 or a
 * negative error. */
WSFRAME_AMD_EXPORT int websocketframeStreamDecodeDevice(unsigned char* d_buf, unsigned long long len,
                                                        unsigned int max_frames, WebsocketFrameDesc_t* d_desc,
                                                        WebsocketSegResult_t* d_res, void* hip_stream);

/* Last HIP error string of the calling thread's most recent failed call ("" if none). */
WSFRAME_AMD_EXPORT const char* websocketframeGpuLastError(void);

/* Launch tuning knobs (for in-process A/B measurement; defaults are the tuned
 * configuration; every value yields bit-identical results, each one is parity-tested in
 * tests/test_gpu_options.py): "path" (-1 auto, 1 walker, 3 piece, 4 segfuse), "scan_alpha"
 * (the piece path's segment walk: 1 switches to alphabet speculation over the lengths seen so far
 * once lengths keep changing, 0 stride speculation only), "piece_lds"
 * (unused dynamic LDS per unmask block:
 * caps its blocks per CU; 0 = the CU's LDS / 7 when the previous call on the stream advised
 * frames of one length <= 16 KiB, / 6 for longer ones, and without advice / 7 for batches with
 * at least one segment per 8 pieces of 16 KiB, else / 6), "piece_win" (0..6: log2 of the windows the
 * unmask kernel streams side by side; -1 default: 2 for batches of >= 32 GiB, and of >= 16 GiB that the
 * previous call on the stream advised as frames of one length, else 1), "seg_win" (0..3: log2 of the windows
 * the segment kernels stream side by side; -1 default: 4 windows for the segment decode, 8 for the
 * fused reassembly; fewer below 256 segments per window), "reasm_path" (0 auto, 1 fused, 2 three-kernel), "reasm_cfg" (0..2: the
 * fused kernel's window/occupancy), "enc_front" (encode: 1 tile-scan front with the edge
 * chunks before the copy, 0 hipcub scan and an edge kernel after it), "host_chunk_mb",
 * "stream_rw" / "stream_rw_cmax" / "stream_rounds" / "stream_plink" (raw stream:
 * chunk-parallel walk 1 linked on the device, 2 eager calls linked by the host, 0 one wavefront;
 * log2 of its largest chunk 16..26, pass rounds of a captured call 1..64, a captured
 * call's chunk records linked in parallel 0/1), "stream_split" / "stream_split2" / "stream_split_wait" /
 * "stream_c0" / "stream_c1" / "stream_side_prio" (raw stream, eager device-planned walk: the unmask's first launch takes this
 * many 256ths of the pieces, 0..255, default 8, 0 = one launch, while the walk of the stream past them runs
 * beside it on a side stream, its last part in chunks of twice the largest chunk;
 * that walk starts after the plan 0, after the first part's owner walks 1 or its emit 2; the first
 * part's chunks are that chunk >> 0..6, default 3; "stream_split2": a second cut in 256ths of the pieces
 * past "stream_split", default 48, 0 = two parts — a middle part, in chunks of that chunk >> "stream_c1"
 * (default 2); "stream_side_prio": the side stream's priority, 0
 * default (default), 1 least, 2 greatest); "stream_split_capture" (0/1, default 1: captured calls
 * split too, the side stream becoming a graph branch; 0 = captured calls take one launch), "stream_win" (-1..6: log2 of the piece windows of a raw-stream
 * call's unmask launches, default 2 = four; -1 the batch rule of "piece_win"), "k2_timing" (see
 * websocketframeGpuGetStat). Options are atomics read once per call. Returns 0, or -1 for an
 * unknown name or a value out of range. */
WSFRAME_AMD_EXPORT int websocketframeGpuSetOption(const char* name, long long value);

/* Counters (diagnostics): "workspace_bytes" (device bytes held
 * in workspace slots), and of the calling process's most recent call: "stream_rw_chunks"
 * (chunks of a long stream written from the chunk-parallel walk's records),
 * "stream_rw_chunk_walks" (chunks it had to walk with one wavefront), "stream_skips" (eager raw-stream
 * calls since load that skipped the pass rounds because the previous chunk walk on the stream saw
 * lengths that keep changing), "stream_splits" (raw-stream calls since load whose unmask
 * ran as two launches beside the split walk, option "stream_split"), "capture_adoptions" (graph captures since load that took over the
 * workspace slot of a destroyed graph whose replays had all finished), "capture_adoption_refusals" (captures
 * since load that passed over such a slot because a replay of its graph was still queued), "k2_windows" (the
 * piece windows of the most recent unmask launch: 1 << the "piece_win" rule's choice); with the option
 * "k2_timing" set, "k2_ns" / "k2_calls" (the summed duration and count of the piece
 * path's unmask launches since the option was set, from HIP events around each launch;
 * reading them waits for those launches). Returns 0, or -1 for an unknown name. */
WSFRAME_AMD_EXPORT int websocketframeGpuGetStat(const char* name, unsigned long long* value);

/* ---- Part 2b: fused decode + fragmented-message reassembly -- */

/* One reassembled message body in the output buffer. 32 bytes. */
typedef struct WebsocketMsgDesc_t {
    unsigned long long out_off;   /* body offset from d_out */
    unsigned long long len;       /* body length = sum of its frames' datalen in this batch */
    unsigned int first_frame;     /* its first frame's index among the segment's descriptors */
    unsigned int n_frames;        /* its frames in this batch */
    unsigned int complete;        /* 1: closed by a FIN frame (delivered); 0: still open at the segment end */
    unsigned int continued;       /* 1: continues a message left open by an earlier batch (d_open) */
} WebsocketMsgDesc_t;

/* Decode every segment exactly as websocketframeBatchDecodeDevice (same descriptors and
 * results; slots s*max_frames), then deliver messages as the reactor's stream hook does
 * with websocket glue: the unmasked body of every consumed frame joins
 * the connection's pending message, and a FIN frame closes it — the message body is the
 * concatenation of its frames' bodies (a FIN frame with nothing pending is one message).
 * Bodies are gathered, unmasked, back to back from d_out + (d_out_off ? d_out_off[s]
 * : d_seg_off[s]) (room for seg_len[s] bytes each); the wire buffer is only read. Message
 * descriptors of segment s are d_msg[s*max_frames + i], i < d_nmsg[s]. d_open (optional,
 * one byte per segment, in/out): 1 = a message is pending from the previous batch.
 * Asynchronous on hip_stream; returns 0 or a negative launch error. */
WSFRAME_AMD_EXPORT int websocketframeBatchReassembleDevice(const unsigned char* d_buf, unsigned long long buflen,
                                                           const unsigned long long* d_seg_off,
                                                           const unsigned long long* d_seg_len, unsigned int nseg,
                                                           unsigned int max_frames, WebsocketFrameDesc_t* d_desc,
                                                           WebsocketSegResult_t* d_res, unsigned char* d_out,
                                                           const unsigned long long* d_out_off,
                                                           WebsocketMsgDesc_t* d_msg, unsigned int* d_nmsg,
                                                           unsigned char* d_open, void* hip_stream);

/* The same with the stream hook's fragment-cache limit (NetChannel_t.readcache_max_size,
 * net_reactor.h:100; 0 = unlimited, as websocketframeBatchReassembleDevice): a frame that is
 * cached (one arriving while a message is pending, or a non-FIN one) and whose body would
 * take the pending message's cached bytes past the limit stops its segment with
 * WEBSOCKET_SEG_ERR_CACHE_OVERFLOW (net_channel_ex.c:129-135). d_cached (optional, one u32
 * per segment, in/out): the pending message's cached bytes, counted as the reference's u32
 * StreamTransportCtx_t.cache_recv_bytes (transport_ctx.c:179-201); 0 whenever d_open is 0. */
WSFRAME_AMD_EXPORT int websocketframeBatchReassembleDeviceEx(const unsigned char* d_buf, unsigned long long buflen,
                                                             const unsigned long long* d_seg_off,
                                                             const unsigned long long* d_seg_len, unsigned int nseg,
                                                             unsigned int max_frames, WebsocketFrameDesc_t* d_desc,
                                                             WebsocketSegResult_t* d_res, unsigned char* d_out,
                                                             const unsigned long long* d_out_off,
                                                             WebsocketMsgDesc_t* d_msg, unsigned int* d_nmsg,
                                                             unsigned char* d_open, unsigned int readcache_max_size,
                                                             unsigned int* d_cached, void* hip_stream);

/* ---- Part 2c: batch encode + client masking -------------- */

/* One frame to emit. The header is exactly websocketframeEncode's
 * (websocketframe.c:167-202); with `masked` set the MASK bit and the 4 key bytes
 * follow it (RFC 6455 §5.2-5.3, client-to-server frames — the reference's encoder
 * never masks) and the payload is XORed with the key. 24 bytes, 8-B aligned. */
typedef struct WebsocketEncodeDesc_t {
    unsigned long long src_off;   /* payload offset in d_src */
    unsigned long long len;       /* payload length (datalen) */
    unsigned int mask_key;        /* key bytes in wire order: byte i = (mask_key >> 8*i) & 0xFF */
    unsigned char type;           /* opcode (websocketframeEncode's type) */
    unsigned char is_fin;         /* websocketframeEncode's is_fin */
    unsigned char prev_is_fin;    /* websocketframeEncode's prev_is_fin */
    unsigned char masked;         /* 1: client frame (MASK + key + XORed payload) */
} WebsocketEncodeDesc_t;

/* Encode nframes frames back to back into d_dst, asynchronously on hip_stream.
 * d_wire_off (device, nframes + 1 u64) receives each frame's wire offset and, last,
 * the total wire length. Bytes past dst_capacity are never written: size d_dst
 * with Σ (len + 14) or read d_wire_off[nframes] first. d_src and d_dst must not
 * overlap. Returns 0 or a negative launch error. */
WSFRAME_AMD_EXPORT int websocketframeBatchEncodeDevice(const unsigned char* d_src,
                                                       const WebsocketEncodeDesc_t* d_frames, unsigned int nframes,
                                                       unsigned char* d_dst, unsigned long long dst_capacity,
                                                       unsigned long long* d_wire_off, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif

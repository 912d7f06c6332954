/*
 * wsframe_amd_channel.h — the reactor-side plugin glue of libwsframe_amd.so.
 *
 * The reference calls websocketframeDecode from user glue registered as
 * NetChannelExProc_t.on_decode (inc/component/net_channel_ex.h:22-23); that glue fills a
 * NetChannelInbufDecodeResult_t (:10-20) which the stream hook on_read_stream
 * (src/component/net_channel_ex.c:110-157) turns into on_recv deliveries, caching
 * fragments until a FIN frame (transport_ctx.c:179-201). This header ships that glue,
 * so a reference application registers it without writing any:
 *
 *   NetChannelExProc_t proc = { websocketframeOnDecode, my_on_recv, NULL, NULL };
 *
 * websocketframeOnDecode decodes one frame in host memory (Part 1 of wsframe_amd.h);
 * websocketframeOnDecodeBatch replays the per-frame results of a GPU batch decode
 * (websocketframeBatchDecodeHost / -Device + copy-back) to the same hook, one
 * descriptor per call, so the reactor loop (net_reactor.c:515-526) runs unchanged on
 * an inbuf the GPU has already unmasked.
 *
 * Both fill the result exactly as the reference glue does:
 *   ret < 0  -> err = 1          ret == 0 -> incomplete = 1
 *   ret > 0  -> decodelen = ret, bodyptr = data, bodylen = (unsigned int)datalen,
 *               fragment_eof = is_fin, pktype = NETPACKET_FRAGMENT (6, transport_ctx.h:11-18)
 * NETPACKET_FRAGMENT (nonzero, != NETPACKET_FIN) routes every frame through the fragment
 * cache, so a FIN frame closes the connection's pending message (net_channel_ex.c:126-153).
 */
#ifndef UTIL_AMD_WSFRAME_AMD_CHANNEL_H
#define UTIL_AMD_WSFRAME_AMD_CHANNEL_H

#include <stddef.h>

#include "wsframe_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

struct NetChannel_t;
struct NetChannelInbufDecodeResult_t;

/* Layout-identical to the reference's NetChannelInbufDecodeResult_t
 * (inc/component/net_channel_ex.h:10-20; checked by tests/c/channel_layout.c against the
 * reference header). The glue entry points take the reference's struct tag, so they can be
 * assigned to NetChannelExProc_t.on_decode without a cast. */
typedef struct WebsocketInbufDecodeResult_t {
    char err;
    char incomplete;
    char fragment_eof;
    char pktype;
    char ignore;
    unsigned int pkseq;
    unsigned int decodelen;
    unsigned int bodylen;
    unsigned char* bodyptr;
} WebsocketInbufDecodeResult_t;

#define WEBSOCKET_NETPACKET_FRAGMENT 6 /* NETPACKET_FRAGMENT, inc/datastruct/transport_ctx.h:11-18 */

/* NetChannelExProc_t.on_decode: one websocketframeDecode on buf[0, len) (unmasks in place).
 * `result` must be zeroed by the caller, as on_read_stream does (net_channel_ex.c:112). */
WSFRAME_AMD_EXPORT void websocketframeOnDecode(struct NetChannel_t* channel, unsigned char* buf, size_t len,
                                               struct NetChannelInbufDecodeResult_t* result);

/* Per-connection replay state of one decoded segment (host copies of its descriptors and
 * result). inbuf = the connection's inbuf holding the segment's bytes as the GPU left them
 * (decoded), inbuf[0] = batch byte seg_off. */
typedef struct WebsocketBatchCursor_t {
    const WebsocketFrameDesc_t* desc; /* the segment's descriptors, res.n_frames of them */
    WebsocketSegResult_t res;         /* the segment's result */
    unsigned long long seg_off;       /* batch offset of inbuf[0] (descriptor offsets are batch offsets) */
    unsigned char* inbuf;             /* where the reactor loop reads the segment */
    unsigned int next;                /* next descriptor to hand out (start at 0) */
} WebsocketBatchCursor_t;

/* on_decode from a batch: the next descriptor of `cursor`, which must describe the frame at
 * buf (buf == inbuf + frame_off - seg_off; else err = 1: the loop left the batch's walk).
 * Past the last descriptor, by the segment's stop reason: OK -> incomplete = 1 (an
 * incomplete tail: the reactor keeps it, net_reactor.c:536-539, and it leads the next
 * read's segment, which starts at m_inbuf[0]); MAX_FRAMES -> the frame at buf is decoded on
 * the host (websocketframeOnDecode), so a short descriptor capacity never stalls a
 * connection; ERR_LEN_WRAP / ERR_DECODE -> err = 1 (the channel is closed, :518-520).
 * Cursor-based: call it from an on_decode that finds the cursor (e.g. through
 * NetChannel_t.userdata); one cursor per read (recv for every readable
 * channel, one batch over their whole m_inbuf, then each channel's on_read loop). */
WSFRAME_AMD_EXPORT void websocketframeOnDecodeBatch(WebsocketBatchCursor_t* cursor, unsigned char* buf, size_t len,
                                                    struct NetChannelInbufDecodeResult_t* result);

#ifdef __cplusplus
}
#endif

#endif

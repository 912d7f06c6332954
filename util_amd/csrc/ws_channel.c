/*
 * ws_channel.c — the NetChannelExProc_t.on_decode glue (include/wsframe_amd_channel.h):
 * how the reference's stream hook (src/component/net_channel_ex.c:110-157) consumes
 * websocketframeDecode's results, for one frame in host memory or replayed from a GPU
 * batch's descriptors.
 */
#include "../../include/wsframe_amd_channel.h"

static void fill(WebsocketInbufDecodeResult_t* r, int ret, unsigned char* data, unsigned long long datalen, int is_fin) {
    if (ret < 0) { r->err = 1; return; }                 /* net_channel_ex.c:116-118 */
    if (ret == 0) { r->incomplete = 1; return; }         /* :119-121 */
    r->decodelen = (unsigned int)ret;
    r->bodyptr = data;
    r->bodylen = (unsigned int)datalen;                  /* the struct's field is 32-bit (net_channel_ex.h:18) */
    r->fragment_eof = (char)is_fin;
    r->pktype = WEBSOCKET_NETPACKET_FRAGMENT;
}

void websocketframeOnDecode(struct NetChannel_t* channel, unsigned char* buf, size_t len,
                            struct NetChannelInbufDecodeResult_t* result) {
    unsigned char* data = 0;
    unsigned long long datalen = 0;
    int is_fin = 0, type = 0;
    int ret = websocketframeDecode(buf, (unsigned long long)len, &data, &datalen, &is_fin, &type);
    (void)channel;
    fill((WebsocketInbufDecodeResult_t*)result, ret, data, datalen, is_fin);
}

void websocketframeOnDecodeBatch(WebsocketBatchCursor_t* cur, unsigned char* buf, size_t len,
                                 struct NetChannelInbufDecodeResult_t* result) {
    WebsocketInbufDecodeResult_t* r = (WebsocketInbufDecodeResult_t*)result;
    const WebsocketFrameDesc_t* d;
    (void)len;
    if (!cur) { r->incomplete = 1; return; }
    if (cur->next >= cur->res.n_frames) {
        /* past the batch's frames: the reactor loop (net_reactor.c:515-526) goes on exactly as
         * it would have without the GPU */
        if (cur->res.status == WEBSOCKET_SEG_MAX_FRAMES) {
            /* descriptor capacity ran out with frames left: decode them here, one per call */
            websocketframeOnDecode(0, buf, len, result);
        } else if (cur->res.status == WEBSOCKET_SEG_ERR_LEN_WRAP || cur->res.status == WEBSOCKET_SEG_ERR_DECODE) {
            r->err = 1;                                   /* fenced wrap (the reference: UB) / ret < 0 */
        } else {
            r->incomplete = 1;                            /* an incomplete tail: kept for the next read */
        }
        return;
    }
    d = cur->desc + cur->next;
    if (buf != cur->inbuf + (d->frame_off - cur->seg_off)) { r->err = 1; return; }
    cur->next++;
    fill(r, d->ret, d->data_off == WEBSOCKET_DATA_OFF_NULL ? 0 : cur->inbuf + (d->data_off - cur->seg_off),
         d->datalen, d->is_fin);
}

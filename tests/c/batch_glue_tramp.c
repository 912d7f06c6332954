/* Test trampoline: NetChannelExProc_t.on_decode replaying one batch's descriptors through
 * websocketframeOnDecodeBatch (include/wsframe_amd_channel.h). The cursor's inbuf is the
 * buffer of the first on_decode call (the start of the channel's inbuf). */
#include "wsframe_amd_channel.h"

static WebsocketBatchCursor_t g_cur;

void tramp_set(const WebsocketFrameDesc_t* desc, unsigned int n_frames, unsigned long long consumed, int status) {
    g_cur.desc = desc;
    g_cur.res.consumed = consumed;
    g_cur.res.n_frames = n_frames;
    g_cur.res.status = status;
    g_cur.seg_off = 0;
    g_cur.inbuf = 0;
    g_cur.next = 0;
}

void tramp_on_decode(struct NetChannel_t* channel, unsigned char* buf, size_t len,
                     struct NetChannelInbufDecodeResult_t* result) {
    (void)channel;
    if (!g_cur.inbuf) g_cur.inbuf = buf;
    websocketframeOnDecodeBatch(&g_cur, buf, len, result);
}

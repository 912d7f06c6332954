/*
 * reactor_harness.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Runs the REFERENCE's own rx stack on a byte stream: NetReactor_handle
 * (src/component/net_reactor.c:1073-1169) → reactor_stream_readev (:465-545, the
 * per-frame loop :515-526) → the stream hook on_read_stream
 * (src/component/net_channel_ex.c:110-157: fragment cache, check_cache_overflow :45-53,
 * streamtransportctxCacheRecvPacket/MergeRecvPacket src/datastruct/transport_ctx.c
 * :179-201, channel_merge_packet_handler/merge_packet :55-108) → on_recv.
 * The reactor, channel, transport and sysapi code are compiled from the reference
 * sources where they lie (oracle/Makefile `ref`, outputs only into oracle/_ref/).
 *
 * The stream is written into one end of an AF_UNIX socketpair in `chunk`-byte writes
 * (so frames are split across recv() calls at arbitrary points) and the other end is a
 * NET_CHANNEL_SIDE_SERVER channel opened with NetChannel_open_with_fd (:1206-1248),
 * wired with NetChannelEx_get_hook(side, SOCK_STREAM) (:616-619) + NetChannelEx_init
 * (:631-654) the way a user of the library does it.
 *
 * on_decode is either the websocket glue below (pktype NETPACKET_FRAGMENT,
 * fragment_eof = is_fin, bodylen = (unsigned int)datalen) around a websocketframeDecode
 * passed in by pointer (the reference's, from oracle/_ref/libwsref.so), or any other
 * on_decode passed in by pointer (libwsframe_amd.so's websocketframeOnDecode: the
 * drop-in check). Every on_recv message is recorded.
 */
#include <errno.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>
#include <fcntl.h>

#include "component/net_channel_ex.h"
#include "component/net_reactor.h"

typedef int (*decode_fn)(unsigned char* buf, unsigned long long len, unsigned char** data,
                         unsigned long long* datalen, int* is_fin, int* type);
typedef void (*on_decode_fn)(NetChannel_t* channel, unsigned char* buf, size_t len,
                             NetChannelInbufDecodeResult_t* result);

typedef struct Run {
    decode_fn decode;
    unsigned char* out;
    unsigned long long out_cap, out_len;
    unsigned long long* msg_len;
    unsigned int max_msgs, n_msgs;
    unsigned long long consumed, frames;
    int detached, detach_error, overrun;
    const NetChannelExHookProc_t* hook;
} Run;

static Run* g_run;   /* one run at a time (the reference callbacks carry no user pointer we own) */

/* the websocket glue a user of the reference writes */
static void ws_glue(NetChannel_t* channel, unsigned char* buf, size_t len, NetChannelInbufDecodeResult_t* r) {
    unsigned char* data = 0;
    unsigned long long datalen = 0;
    int is_fin = 0, type = 0;
    int ret = g_run->decode(buf, len, &data, &datalen, &is_fin, &type);
    (void)channel;
    if (ret < 0) { r->err = 1; return; }
    if (ret == 0) { r->incomplete = 1; return; }
    r->decodelen = (unsigned int)ret;
    r->bodyptr = data;
    r->bodylen = (unsigned int)datalen;
    r->fragment_eof = (char)is_fin;
    r->pktype = NETPACKET_FRAGMENT;
}

static void rec_recv(NetChannel_t* channel, unsigned char* bodyptr, size_t bodylen, const struct sockaddr* a,
                     socklen_t al) {
    Run* R = g_run;
    (void)channel; (void)a; (void)al;
    if (R->n_msgs >= R->max_msgs || R->out_len + bodylen > R->out_cap) { R->overrun = 1; return; }
    if (bodylen) memcpy(R->out + R->out_len, bodyptr, bodylen);
    R->out_len += bodylen;
    R->msg_len[R->n_msgs++] = bodylen;
}

/* on_read = the stream hook, counting what the reactor loop consumes (net_reactor.c:516-525) */
static int counted_read(NetChannel_t* ch, unsigned char* buf, unsigned int len, long long ts,
                        const struct sockaddr* a, socklen_t al) {
    int r = g_run->hook->on_read(ch, buf, len, ts, a, al);
    if (r > 0) { g_run->consumed += (unsigned int)r; g_run->frames++; }
    return r;
}

static void on_detach(NetChannel_t* ch) {
    g_run->detached = 1;
    g_run->detach_error = ch->detach_error;
    NetChannel_close_ref(ch);
}

/*
 * Returns 0 on success (results in the out-params), < 0 on a harness failure.
 *   wire/len        the byte stream a peer sends on one connection
 *   chunk           bytes per write() (>= 1)
 *   readcache_max   NetChannel_t.readcache_max_size (0 = unlimited, net_reactor.h:100)
 *   decode / glue   glue == NULL: ws_glue around decode; else glue is on_decode
 *   out, msg_len    message bodies back to back, their lengths (max_msgs)
 *   consumed/frames bytes/frames the reactor loop consumed (Σ on_read returns > 0)
 *   detach_error    NetChannel_t.detach_error at detach (0 = still attached at the end)
 *   pending/cached  at the end: fragments still cached (stream_ctx.recvlist non-empty) and
 *                   stream_ctx.cache_recv_bytes (transport_ctx.c:179-201)
 */
__attribute__((visibility("default")))
int ref_reactor_deliver(const unsigned char* wire, unsigned long long len, unsigned int chunk,
                        unsigned int readcache_max, decode_fn decode, on_decode_fn glue,
                        unsigned char* out, unsigned long long out_cap, unsigned long long* msg_len,
                        unsigned int max_msgs, unsigned int* n_msgs, unsigned long long* consumed,
                        unsigned long long* frames, int* detach_error, int* pending, unsigned int* cached) {
    Run R;
    NetChannelProc_t proc;
    NetChannelExProc_t exproc;
    NetChannelExData_t exdata;
    struct NetReactor_t* reactor;
    NetChannel_t* ch;
    NioEv_t ev[16];
    int sp[2], idle = 0, rounds = 0;
    unsigned long long sent = 0;

    memset(&R, 0, sizeof(R));
    R.decode = decode;
    R.out = out; R.out_cap = out_cap; R.msg_len = msg_len; R.max_msgs = max_msgs;
    R.hook = NetChannelEx_get_hook(NET_CHANNEL_SIDE_SERVER, SOCK_STREAM);
    g_run = &R;
    if (chunk == 0) return -1;
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sp)) return -2;
    fcntl(sp[1], F_SETFL, fcntl(sp[1], F_GETFL) | O_NONBLOCK);
    reactor = NetReactor_create();
    if (!reactor) return -3;
    memset(&proc, 0, sizeof(proc));
    proc.on_read = counted_read;
    proc.on_pre_send = R.hook->on_pre_send;
    proc.on_detach = on_detach;
    memset(&exproc, 0, sizeof(exproc));
    exproc.on_decode = glue ? glue : ws_glue;
    exproc.on_recv = rec_recv;
    ch = NetChannel_open_with_fd(NET_CHANNEL_SIDE_SERVER, &proc, sp[0], AF_UNIX, 0);
    if (!ch) return -4;
    NetChannelEx_init(ch, &exdata, &exproc);
    ch->readcache_max_size = readcache_max;
    NetChannel_reg(reactor, ch);

    /* feed the stream; then run the reactor until it has been idle for a few rounds */
    while (!R.detached && (sent < len || idle < 3)) {
        if (sent < len) {
            unsigned long long n = len - sent < chunk ? len - sent : chunk;
            ssize_t w = write(sp[1], wire + sent, (size_t)n);
            if (w > 0) sent += (unsigned long long)w;
            else if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK) break;
        }
        int n = NetReactor_handle(reactor, ev, 16, sent < len ? 0 : 1);
        idle = (n == 0 && sent >= len) ? idle + 1 : 0;
        if (++rounds > 100000000) break;
    }
    *n_msgs = R.n_msgs;
    *consumed = R.consumed;
    *frames = R.frames;
    *detach_error = R.detached ? R.detach_error : 0;
    *pending = ch->stream_ctx.recvlist.head != 0;
    *cached = ch->stream_ctx.cache_recv_bytes;
    if (!R.detached) NetChannel_close_ref(ch);
    close(sp[1]);
    {   /* let the reactor run the channel's free command, then drop it */
        int i;
        for (i = 0; i < 4; ++i) NetReactor_handle(reactor, ev, 16, 0);
    }
    NetReactor_destroy(reactor);
    g_run = 0;
    return R.overrun ? -5 : 0;
}

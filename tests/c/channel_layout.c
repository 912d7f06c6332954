/*
 * channel_layout.c — compiled by tests/test_abi.py (dev container, where the reference
 * headers exist) against the REFERENCE's inc/component/net_channel_ex.h together with
 * include/wsframe_amd_channel.h:
 *   - WebsocketInbufDecodeResult_t has NetChannelInbufDecodeResult_t's exact layout
 *     (net_channel_ex.h:10-20);
 *   - websocketframeOnDecode is assignable to NetChannelExProc_t.on_decode (:22-23) without
 *     a cast (-Werror: no incompatible-pointer warning);
 *   - WEBSOCKET_NETPACKET_FRAGMENT == NETPACKET_FRAGMENT (transport_ctx.h:11-18).
 * Links to libwsframe_amd.so and runs the glue once on a masked frame.
 */
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "component/net_channel_ex.h"
#include "wsframe_amd_channel.h"

#define SAME(f) (offsetof(NetChannelInbufDecodeResult_t, f) == offsetof(WebsocketInbufDecodeResult_t, f))
_Static_assert(sizeof(NetChannelInbufDecodeResult_t) == sizeof(WebsocketInbufDecodeResult_t), "size");
_Static_assert(SAME(err) && SAME(incomplete) && SAME(fragment_eof) && SAME(pktype) && SAME(ignore), "flags");
_Static_assert(SAME(pkseq) && SAME(decodelen) && SAME(bodylen) && SAME(bodyptr), "fields");
_Static_assert(WEBSOCKET_NETPACKET_FRAGMENT == NETPACKET_FRAGMENT, "pktype");

static void on_recv(NetChannel_t* ch, unsigned char* p, size_t n, const struct sockaddr* a, socklen_t al) {
    (void)ch; (void)p; (void)n; (void)a; (void)al;
}

int main(void) {
    NetChannelExProc_t proc = {websocketframeOnDecode, on_recv, NULL, NULL};
    unsigned char f[2 + 4 + 3] = {0x81, 0x83, 1, 2, 3, 4, 'a' ^ 1, 'b' ^ 2, 'c' ^ 3};
    NetChannelInbufDecodeResult_t r;
    memset(&r, 0, sizeof(r));
    proc.on_decode(NULL, f, sizeof(f), &r);
    if (r.err || r.incomplete || r.decodelen != 9 || r.bodylen != 3 || r.bodyptr != f + 6 || !r.fragment_eof ||
        r.pktype != NETPACKET_FRAGMENT || memcmp(r.bodyptr, "abc", 3)) {
        fprintf(stderr, "channel_layout: glue result wrong\n");
        return 1;
    }
    memset(&r, 0, sizeof(r));
    proc.on_decode(NULL, f, 5, &r);
    if (!r.incomplete || r.err) return 1;
    printf("channel_layout ok\n");
    return 0;
}

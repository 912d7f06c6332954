/*
 * drop_in.c — a C caller written against the reference's websocketframe API
 * (inc/crt/protocol/websocketframe.h:42-49), the way reactor glue uses it, linked
 * against libwsframe_amd.so instead of websocketframe.c. Host symbols only (no GPU).
 * Built and run by tests/test_abi.py: against include/wsframe_amd.h, and (dev container)
 * against the REFERENCE's own header inc/crt/protocol/websocketframe.h
 * (-DWS_API_HEADER='"crt/protocol/websocketframe.h"' -I /root/reference/inc): a source
 * file written for the reference compiles unchanged and links to libwsframe_amd.so.
 *
 * 1. encode a header with websocketframeEncode, mask the payload like a client, then
 *    decode it with the reference's per-frame loop (net_reactor.c:515-526) and check
 *    the out-params and the unmasked bytes;
 * 2. RFC 6455 §1.3 handshake sample through websocketframeComputeSecAccept and the
 *    response encoders; a request built from WEBSOCKET_SIMPLE_HTTP_HANDSHAKE_REQUEST_FMT
 *    (websocketframe.h:21-36) parsed back by websocketframeDecodeHandshakeRequest.
 * Prints "drop_in ok" and exits 0 on success.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef WS_API_HEADER
#define WS_API_HEADER "wsframe_amd.h"
#endif
#include WS_API_HEADER

static int fail(const char* what) {
    fprintf(stderr, "drop_in: %s\n", what);
    return 1;
}

int main(void) {
    unsigned char buf[3 * (14 + 300)];
    unsigned char plain[3][300];
    const unsigned long long lens[3] = {5, 126, 300};
    const unsigned char key[4] = {0x37, 0xfa, 0x21, 0x3d};
    unsigned long long off = 0, i;
    int f;
    for (f = 0; f < 3; ++f) {
        unsigned int hl = websocketframeEncodeHeadLength(lens[f]);
        websocketframeEncode(buf + off, f == 2, f == 0, WEBSOCKET_TEXT_FRAME, lens[f]);
        buf[off + 1] |= 0x80;                                  /* client frame: MASK + key */
        memcpy(buf + off + hl, key, 4);
        for (i = 0; i < lens[f]; ++i) {
            plain[f][i] = (unsigned char)('a' + (i * 7 + f) % 26);
            buf[off + hl + 4 + i] = plain[f][i] ^ key[i % 4];
        }
        off += hl + 4 + lens[f];
    }
    /* the reactor's loop over one inbuf */
    {
        unsigned long long pos = 0;
        int n = 0;
        while (pos < off) {
            unsigned char* data;
            unsigned long long datalen;
            int is_fin, type;
            int r = websocketframeDecode(buf + pos, off - pos, &data, &datalen, &is_fin, &type);
            if (r < 0) return fail("decode error");
            if (r == 0) break;
            if (datalen != lens[n] || memcmp(data, plain[n], datalen)) return fail("payload");
            if (is_fin != (n == 2)) return fail("fin");
            if (type != (n == 0 ? WEBSOCKET_TEXT_FRAME : WEBSOCKET_CONTINUE_FRAME)) return fail("type");
            pos += (unsigned int)r;
            ++n;
        }
        if (n != 3 || pos != off) return fail("frame count");
    }
    /* RFC 6455 §1.3: "dGhlIHNhbXBsZSBub25jZQ==" -> "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=" */
    {
        char acc[60];
        const char* k = "dGhlIHNhbXBsZSBub25jZQ==";
        char resp[162];
        char* r2;
        if (!websocketframeComputeSecAccept(k, (unsigned int)strlen(k), acc)) return fail("sec accept");
        if (strcmp(acc, "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=")) return fail("sec accept value");
        if (!websocketframeEncodeHandshakeResponse(acc, (unsigned int)strlen(acc), resp)) return fail("response");
        if (!strstr(resp, "Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=")) return fail("response text");
        r2 = websocketframeEncodeHandshakeResponseWithProtocol(acc, (unsigned int)strlen(acc), "chat", 4);
        if (!r2 || !strstr(r2, "Sec-WebSocket-Protocol: chat")) return fail("protocol response");
        websocketframeFreeString(r2);
    }
    /* the request templates (websocketframe.h:21-36) round-trip through the request parser */
    {
        char req[512];
        const char *sk = NULL, *sp = NULL;
        unsigned int skl = 0, spl = 0;
        snprintf(req, sizeof(req), WEBSOCKET_SIMPLE_HTTP_HANDSHAKE_REQUEST_WITH_PROTOCOL_FMT, "/chat",
                 "dGhlIHNhbXBsZSBub25jZQ==", "superchat");
        if (!websocketframeDecodeHandshakeRequest(req, (unsigned int)strlen(req), &sk, &skl, &sp, &spl))
            return fail("request parse");
        if (skl != 24 || strncmp(sk, "dGhlIHNhbXBsZSBub25jZQ==", 24)) return fail("request key");
        if (spl != 9 || strncmp(sp, "superchat", 9)) return fail("request protocol");
        snprintf(req, sizeof(req), WEBSOCKET_SIMPLE_HTTP_HANDSHAKE_REQUEST_FMT, "/", "x3JJHMbDL1EzLkh9GBhXDw==");
        if (!websocketframeDecodeHandshakeRequest(req, (unsigned int)strlen(req), &sk, &skl, &sp, &spl))
            return fail("request parse 2");
        if (skl != 24 || strncmp(sk, "x3JJHMbDL1EzLkh9GBhXDw==", 24)) return fail("request key 2");
    }
    printf("drop_in ok\n");
    return 0;
}

/*
 * ws_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference
 * hot path, used as the parity checker by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg. Never linked into or called by the product
 * (util_amd/ / libwsframe_amd.so).
 *
 * Pinned: tests/test_oracle_golden.py checks every function here against
 * golden vectors produced by the reference itself, compiled from
 * /root/reference by oracle/Makefile into oracle/_ref/ (tests/golden/
 * make_golden.py). Deliberately the reference's scalar algorithm (one byte per
 * iteration, `i % 4`), compiled with the reference flags -O2 -fwrapv
 * -fno-strict-aliasing (makefile:5,31), so it doubles as the "port" CPU
 * baseline.
 *
 * Reference map (file:line relative to hujianzhe/util):
 *   ws_oracle_read_be          memReadBE16/BE64   src/datastruct/memfunc.c:80-84,104-110,136-142
 *   ws_oracle_decode           websocketframeDecode   src/crt/protocol/websocketframe.c:112-165
 *   ws_oracle_encode_headlen   websocketframeEncodeHeadLength   websocketframe.c:167-174
 *   ws_oracle_encode           websocketframeEncode   websocketframe.c:176-202
 *   ws_oracle_decode_segments  reactor rx loop   src/component/net_reactor.c:515-526
 *   ws_oracle_sha1 / _base64 / _sec_accept   websocketframe.c:16-32, sha1.c:59-184, base64.c:13-43
 */
#include <stdlib.h>
#include <string.h>
#include "../include/wsframe_amd.h"

#define ORACLE_API __attribute__((visibility("default")))

/* memfunc.c:80-84 macro_READ_BE: most significant byte first, byte by byte */
static unsigned long long ws_oracle_read_be(const unsigned char* p, int n) {
    unsigned long long v = 0;
    int i;
    for (i = 0; i < n; ++i) v = (v << 8) | p[i];
    return v;
}

/* websocketframe.c:112-165 */
ORACLE_API int ws_oracle_decode(unsigned char* buf, unsigned long long len, unsigned char** data,
                                unsigned long long* datalen, int* is_fin, int* type) {
    unsigned int ext = 0, mask = 0;               /* :116 */
    unsigned long long plen;
    unsigned char* payload;
    if (len < 2) return 0;                        /* :121-122 */
    mask = (buf[1] >> 7) ? 4u : 0u;               /* :126-127 */
    plen = buf[1] & 0x7f;                         /* :129 */
    if (plen == 126) ext = 2;                     /* :134-135 */
    else if (plen == 127) ext = 8;                /* :140-141 */
    if (len < 2u + ext + mask) return 0;          /* :131,136,142 */
    if (ext) plen = ws_oracle_read_be(buf + 2, (int)ext); /* :138,144 */
    /* :149 — unsigned 64-bit sum, may wrap */
    if (len < (unsigned long long)(2u + ext + mask) + plen) return 0;
    payload = buf + 2 + ext + mask;               /* :152 */
    if (mask) {                                   /* :153-158, the scalar hot loop */
        unsigned long long i;
        unsigned char* key = buf + 2 + ext;
        for (i = 0; i < plen; ++i) payload[i] ^= key[i % 4];
    }
    *is_fin = buf[0] >> 7;                        /* :124,160 */
    *type = buf[0] & 0x0f;                        /* :125,161 */
    *datalen = plen;                              /* :162 */
    *data = plen ? payload : NULL;                /* :163 */
    return (int)((unsigned long long)(2u + ext + mask) + plen); /* :164, truncating */
}

/* websocketframe.c:167-174 */
ORACLE_API unsigned int ws_oracle_encode_headlen(unsigned long long datalen) {
    return datalen < 126 ? 2u : (datalen <= 0xffff ? 4u : 10u);
}

/* websocketframe.c:176-202 */
ORACLE_API void ws_oracle_encode(void* headbuf, int is_fin, int prev_is_fin, int type,
                                 unsigned long long datalen) {
    unsigned char* h = (unsigned char*)headbuf;
    int i;
    if (prev_is_fin) h[0] = (unsigned char)(is_fin ? (type | 0x80) : type);
    else h[0] = (unsigned char)(is_fin ? 0x80 : 0x00);
    if (datalen < 126) {
        h[1] = (unsigned char)datalen;
    } else if (datalen <= 0xffff) {
        h[1] = 126;
        h[2] = (unsigned char)(datalen >> 8);
        h[3] = (unsigned char)datalen;
    } else {
        h[1] = 127;
        for (i = 0; i < 8; ++i) h[2 + i] = (unsigned char)(datalen >> (56 - 8 * i));
    }
}

/* Decode one frame into a descriptor, mirroring websocketframeDecode, with the
 * one fence the batch API defines: a MASKED frame whose u64 length sum wraps
 * (websocketframe.c:149) would make the reference unmask past the buffer end
 * (undefined behaviour); report WEBSOCKET_SEG_ERR_LEN_WRAP instead.
 * Returns 1 if ret was produced (*ret valid), 0 for the fenced case. */
static int ws_oracle_decode_one(unsigned char* base, unsigned long long off, unsigned long long avail,
                                WebsocketFrameDesc_t* d, int* ret) {
    unsigned char* p = base + off;
    unsigned char* data = NULL;
    unsigned long long datalen = 0;
    int fin = 0, type = 0;
    if (avail >= 2) {
        unsigned int ext = (p[1] & 0x7f) == 126 ? 2u : ((p[1] & 0x7f) == 127 ? 8u : 0u);
        unsigned int mask = (p[1] >> 7) ? 4u : 0u;
        if (mask && avail >= 2u + ext + mask) {
            unsigned long long plen = ext ? ws_oracle_read_be(p + 2, (int)ext) : (unsigned long long)(p[1] & 0x7f);
            unsigned long long tot = (unsigned long long)(2u + ext + mask) + plen;
            if (tot < plen && avail >= tot) return 0; /* wrapped and would be "complete" */
        }
    }
    *ret = ws_oracle_decode(p, avail, &data, &datalen, &fin, &type);
    if (*ret != 0) {
        d->frame_off = off;
        d->data_off = data ? (unsigned long long)(data - base) : WEBSOCKET_DATA_OFF_NULL;
        d->datalen = datalen;
        d->ret = *ret;
        d->is_fin = (unsigned char)fin;
        d->type = (unsigned char)type;
        d->masked = (unsigned char)(p[1] >> 7);
        d->hdrlen = (unsigned char)(2 + ((p[1] & 0x7f) == 126 ? 2 : ((p[1] & 0x7f) == 127 ? 8 : 0)) +
                                    ((p[1] >> 7) ? 4 : 0));
    }
    return 1;
}

/* The reactor rx loop (net_reactor.c:515-526) over each segment:
 *   off = 0; while (off < len) { r = decode(buf+off, len-off);
 *     if (r < 0) error; if (r == 0) break; off += r; }
 * Descriptors of segment s start at desc_base ? desc_base[s] : s*max_frames. */
ORACLE_API void ws_oracle_decode_segments(unsigned char* buf, const unsigned long long* seg_off,
                                          const unsigned long long* seg_len, unsigned int nseg,
                                          unsigned int max_frames, const unsigned long long* desc_base,
                                          WebsocketFrameDesc_t* desc, WebsocketSegResult_t* res) {
    unsigned int s;
    for (s = 0; s < nseg; ++s) {
        unsigned long long so = seg_off[s], len = seg_len[s], off = 0;
        WebsocketFrameDesc_t* out = desc + (desc_base ? desc_base[s] : (unsigned long long)s * max_frames);
        unsigned int nf = 0;
        int status = WEBSOCKET_SEG_OK;
        while (off < len) {
            int r = 0;
            WebsocketFrameDesc_t d;
            if (nf >= max_frames) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
            if (!ws_oracle_decode_one(buf, so + off, len - off, &d, &r)) {
                status = WEBSOCKET_SEG_ERR_LEN_WRAP;
                break;
            }
            if (r == 0) break;
            out[nf++] = d;
            if (r < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }
            off += (unsigned int)r;
        }
        res[s].consumed = off;
        res[s].n_frames = nf;
        res[s].status = status;
    }
}

/* ---- handshake: FIPS 180-1 SHA-1 and RFC 4648 base64 ---- */

static unsigned int rol32(unsigned int x, int n) { return (x << n) | (x >> (32 - n)); }

ORACLE_API void ws_oracle_sha1(const unsigned char* msg, unsigned long long n, unsigned char out[20]) {
    unsigned int h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    unsigned long long total = ((n + 8) / 64 + 1) * 64, blk, bits = n * 8;
    unsigned char* m = (unsigned char*)calloc((size_t)total, 1);
    int i;
    memcpy(m, msg, (size_t)n);
    m[n] = 0x80;
    for (i = 0; i < 8; ++i) m[total - 1 - i] = (unsigned char)(bits >> (8 * i));
    for (blk = 0; blk < total; blk += 64) {
        unsigned int w[80], a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f, k, t;
        for (i = 0; i < 16; ++i)
            w[i] = ((unsigned int)m[blk + 4 * i] << 24) | ((unsigned int)m[blk + 4 * i + 1] << 16) |
                   ((unsigned int)m[blk + 4 * i + 2] << 8) | m[blk + 4 * i + 3];
        for (i = 16; i < 80; ++i) w[i] = rol32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        for (i = 0; i < 80; ++i) {
            if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
            else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
            t = rol32(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol32(b, 30); b = a; a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }
    free(m);
    for (i = 0; i < 20; ++i) out[i] = (unsigned char)(h[i / 4] >> (24 - 8 * (i % 4)));
}

/* base64.c:13-43 behaviour: RFC 4648 alphabet, '=' padding, NUL terminated */
ORACLE_API unsigned long long ws_oracle_base64(const unsigned char* src, unsigned long long n, char* dst) {
    static const char al[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    unsigned long long i, o = 0;
    for (i = 0; i + 2 < n; i += 3) {
        unsigned int v = ((unsigned int)src[i] << 16) | ((unsigned int)src[i + 1] << 8) | src[i + 2];
        dst[o++] = al[v >> 18]; dst[o++] = al[(v >> 12) & 63]; dst[o++] = al[(v >> 6) & 63]; dst[o++] = al[v & 63];
    }
    if (i < n) {
        unsigned int v = (unsigned int)src[i] << 16;
        if (i + 1 < n) v |= (unsigned int)src[i + 1] << 8;
        dst[o++] = al[v >> 18];
        dst[o++] = al[(v >> 12) & 63];
        dst[o++] = (i + 1 < n) ? al[(v >> 6) & 63] : '=';
        dst[o++] = '=';
    }
    dst[o] = 0;
    return o;
}

/* websocketframe.c:16-32: base64(SHA1(key || RFC 6455 GUID)) */
ORACLE_API char* ws_oracle_sec_accept(const char* key, unsigned int keylen, char out[60]) {
    static const char guid[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
    unsigned char dg[20];
    unsigned char* m = (unsigned char*)malloc(keylen + sizeof(guid) - 1);
    if (!m) return NULL;
    memcpy(m, key, keylen);
    memcpy(m + keylen, guid, sizeof(guid) - 1);
    ws_oracle_sha1(m, keylen + sizeof(guid) - 1, dg);
    free(m);
    ws_oracle_base64(dg, 20, out);
    return out;
}

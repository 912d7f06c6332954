/*
 * batch_host.c — a plain C caller of the GPU batch API (no Python, no torch): the rx
 * inbufs of many connections in one host buffer, decoded on the GPU with
 * websocketframeBatchDecodeHost, and checked against the reference's per-frame loop
 * (net_reactor.c:515-526 over websocketframeDecode) run on a copy with the host symbols.
 * Built and run by tests/test_gpu_c_api.py on the GPU box.
 * Prints "batch_host ok <frames>" and exits 0 on success.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wsframe_amd.h"

#define NSEG 2000
#define MAXF 8

static unsigned long long rng_state = 0x9E3779B97F4A7C15ull;
static unsigned int rnd(void) {                                 /* xorshift64* */
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (unsigned int)((rng_state * 0x2545F4914F6CDD1Dull) >> 32);
}

int main(void) {
    static const unsigned long long lens[] = {0, 1, 15, 16, 17, 125, 126, 1000, 4096, 70000};
    unsigned long long cap = (unsigned long long)NSEG * MAXF * (70000 + 14) / 4 + 64, pos = 0;
    unsigned char* buf = (unsigned char*)malloc(cap);
    unsigned long long so[NSEG], sl[NSEG];
    int s, k;
    if (!buf) return 1;
    for (s = 0; s < NSEG; ++s) {
        const int nf = (int)(rnd() % (MAXF + 2));             /* sometimes more than MAXF: MAX_FRAMES */
        pos += rnd() % 8;                                      /* gaps between inbufs */
        so[s] = pos;
        for (k = 0; k < nf; ++k) {
            const unsigned long long n = lens[rnd() % (sizeof lens / sizeof lens[0])];
            const unsigned int hl = websocketframeEncodeHeadLength(n);
            const int masked = (rnd() & 3) != 0;
            unsigned char key[4];
            unsigned long long i;
            if (pos + hl + 4 + n + 64 > cap) break;
            websocketframeEncode(buf + pos, 1, 1, WEBSOCKET_BINARY_FRAME, n);
            for (i = 0; i < 4; ++i) key[i] = (unsigned char)rnd();
            if (masked) { buf[pos + 1] |= 0x80; memcpy(buf + pos + hl, key, 4); }
            pos += hl + (masked ? 4 : 0);
            for (i = 0; i < n; ++i) buf[pos + i] = (unsigned char)rnd();
            pos += n;
        }
        if (rnd() % 4 == 0 && pos > so[s]) pos -= rnd() % (pos - so[s]);   /* incomplete tail */
        sl[s] = pos - so[s];
    }
    {
        const unsigned long long total = pos;
        unsigned char* ref = (unsigned char*)malloc(total + 64);
        WebsocketFrameDesc_t* d = (WebsocketFrameDesc_t*)calloc((size_t)NSEG * MAXF, sizeof *d);
        WebsocketSegResult_t* r = (WebsocketSegResult_t*)calloc(NSEG, sizeof *r);
        unsigned long long frames = 0;
        if (!ref || !d || !r) return 1;
        memcpy(ref, buf, total);
        memset(buf + total, 0, 64);
        if (websocketframeBatchDecodeHost(buf, total, so, sl, NSEG, MAXF, d, r, 0)) {
            fprintf(stderr, "batch_host: %s\n", websocketframeGpuLastError());
            return 1;
        }
        for (s = 0; s < NSEG; ++s) {                           /* the reactor loop, reference semantics */
            unsigned long long off = 0;
            unsigned int nf = 0;
            int status = WEBSOCKET_SEG_OK;
            while (off < sl[s]) {
                unsigned char* data;
                unsigned long long datalen;
                int is_fin, type, rr;
                if (nf >= MAXF) { status = WEBSOCKET_SEG_MAX_FRAMES; break; }
                rr = websocketframeDecode(ref + so[s] + off, sl[s] - off, &data, &datalen, &is_fin, &type);
                if (rr == 0) break;
                {
                    const WebsocketFrameDesc_t* g = d + (size_t)s * MAXF + nf;
                    if (g->frame_off != so[s] + off || g->datalen != datalen || g->ret != rr ||
                        g->is_fin != is_fin || g->type != type ||
                        g->data_off != (data ? (unsigned long long)(data - ref) : WEBSOCKET_DATA_OFF_NULL)) {
                        fprintf(stderr, "batch_host: descriptor %d/%u differs\n", s, nf);
                        return 1;
                    }
                }
                ++nf;
                if (rr < 0) { status = WEBSOCKET_SEG_ERR_DECODE; break; }
                off += (unsigned int)rr;
            }
            if (r[s].consumed != off || r[s].n_frames != nf || r[s].status != status) {
                fprintf(stderr, "batch_host: segment %d result differs\n", s);
                return 1;
            }
            frames += nf;
        }
        if (memcmp(buf, ref, total)) { fprintf(stderr, "batch_host: bytes differ\n"); return 1; }
        printf("batch_host ok %llu\n", frames);
        free(ref); free(d); free(r);
    }
    free(buf);
    return 0;
}

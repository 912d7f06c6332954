/*
 * stream_dev.c — a plain C caller of the raw-stream device API: one connection's inbuf
 * (client frames of changing lengths, a truncated last frame) copied to HBM with the HIP
 * runtime, decoded with websocketframeStreamDecodeDevice, and checked against the
 * reference's per-frame loop (net_reactor.c:515-526 over websocketframeDecode, the host
 * symbols) on a host copy: descriptors, segment result and every byte.
 * Built with gcc against include/wsframe_amd.h and <hip/hip_runtime_api.h> and run by
 * tests/test_gpu_c_api.py on the GPU box. Prints "stream_dev ok <frames>".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "wsframe_amd.h"

#define MAXF 200000u

static unsigned long long rng_state = 0x243F6A8885A308D3ull;
static unsigned int rnd(void) {                                 /* xorshift64* */
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (unsigned int)((rng_state * 0x2545F4914F6CDD1Dull) >> 32);
}

static int fail(const char* what) {
    fprintf(stderr, "stream_dev: %s (%s)\n", what, websocketframeGpuLastError());
    return 1;
}

int main(void) {
    static const unsigned long long lens[] = {0, 1, 7, 125, 126, 1000, 1500, 4096, 20000, 65536, 70000};
    const unsigned long long cap = 24ull << 20;
    unsigned char* buf = (unsigned char*)malloc(cap + 64);
    unsigned char* ref;
    unsigned long long pos = 0, i;
    unsigned int nframes_built = 0;
    unsigned char *d_buf = NULL, *d_desc = NULL, *d_res = NULL;
    WebsocketFrameDesc_t* desc;
    WebsocketSegResult_t res;
    if (!buf) return 1;
    while (1) {                                                 /* client frames, lengths changing */
        const unsigned long long n = lens[rnd() % (sizeof lens / sizeof lens[0])];
        const unsigned int hl = websocketframeEncodeHeadLength(n);
        unsigned char key[4];
        if (pos + hl + 4 + n > cap - 4096) break;
        websocketframeEncode(buf + pos, 1, 1, WEBSOCKET_BINARY_FRAME, n);
        for (i = 0; i < 4; ++i) key[i] = (unsigned char)rnd();
        buf[pos + 1] |= 0x80;
        memcpy(buf + pos + hl, key, 4);
        pos += hl + 4;
        for (i = 0; i < n; ++i) buf[pos + i] = (unsigned char)rnd();
        pos += n;
        ++nframes_built;
    }
    {                                                           /* a truncated last frame */
        const unsigned int hl = websocketframeEncodeHeadLength(3000);
        websocketframeEncode(buf + pos, 1, 1, WEBSOCKET_TEXT_FRAME, 3000);
        buf[pos + 1] |= 0x80;
        memset(buf + pos + hl, 0x5A, 4 + 1000);
        pos += hl + 4 + 1000;
    }
    memset(buf + pos, 0, 64);
    ref = (unsigned char*)malloc(pos + 64);
    desc = (WebsocketFrameDesc_t*)calloc(MAXF, sizeof *desc);
    if (!ref || !desc) return 1;
    memcpy(ref, buf, pos + 64);
    if (hipMalloc((void**)&d_buf, pos + WEBSOCKET_BATCH_PAD) != hipSuccess ||
        hipMalloc((void**)&d_desc, (size_t)MAXF * sizeof *desc) != hipSuccess ||
        hipMalloc((void**)&d_res, sizeof res) != hipSuccess)
        return fail("hipMalloc");
    if (hipMemcpy(d_buf, buf, pos + WEBSOCKET_BATCH_PAD, hipMemcpyHostToDevice) != hipSuccess)
        return fail("hipMemcpy H2D");
    if (websocketframeStreamDecodeDevice(d_buf, pos, MAXF, (WebsocketFrameDesc_t*)d_desc,
                                         (WebsocketSegResult_t*)d_res, NULL))
        return fail("websocketframeStreamDecodeDevice");
    if (hipMemcpy(buf, d_buf, pos, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(desc, d_desc, (size_t)MAXF * sizeof *desc, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&res, d_res, sizeof res, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("hipMemcpy D2H");
    {                                                           /* the reactor loop, reference semantics */
        unsigned long long off = 0;
        unsigned int nf = 0;
        while (off < pos) {
            unsigned char* data;
            unsigned long long datalen;
            int is_fin, type, rr;
            rr = websocketframeDecode(ref + off, pos - off, &data, &datalen, &is_fin, &type);
            if (rr == 0) break;
            {
                const WebsocketFrameDesc_t* g = desc + nf;
                if (g->frame_off != off || g->datalen != datalen || g->ret != rr || g->is_fin != is_fin ||
                    g->type != type ||
                    g->data_off != (data ? (unsigned long long)(data - ref) : WEBSOCKET_DATA_OFF_NULL)) {
                    fprintf(stderr, "stream_dev: descriptor %u differs\n", nf);
                    return 1;
                }
            }
            ++nf;
            if (rr < 0) break;
            off += (unsigned int)rr;
        }
        if (res.consumed != off || res.n_frames != nf || res.status != WEBSOCKET_SEG_OK || nf != nframes_built)
            return fail("segment result");
        if (memcmp(buf, ref, pos)) return fail("bytes");
        printf("stream_dev ok %u\n", nf);
    }
    hipFree(d_buf);
    hipFree(d_desc);
    hipFree(d_res);
    free(buf);
    free(ref);
    free(desc);
    return 0;
}

/*
 * ref_loop.c — TEST INFRASTRUCTURE ONLY. Drives the REFERENCE build
 * (oracle/_ref/libwsref.so, compiled from /root/reference sources) with the
 * reactor's per-frame loop, src/component/net_reactor.c:515-526, so the CPU
 * baseline times the reference's own websocketframeDecode (kind "reference").
 * Linked only into oracle/_ref/libwsref_loop.so.
 */
#include <stddef.h>

int websocketframeDecode(unsigned char* buf, unsigned long long len, unsigned char** data,
                         unsigned long long* datalen, int* is_fin, int* type);

/* returns bytes consumed over all segments; *frames = frames decoded */
__attribute__((visibility("default")))
unsigned long long ref_decode_segments(unsigned char* buf, const unsigned long long* seg_off,
                                       const unsigned long long* seg_len, unsigned int nseg,
                                       unsigned long long* frames) {
    unsigned long long total = 0, nf = 0;
    unsigned int s;
    for (s = 0; s < nseg; ++s) {
        unsigned char* p = buf + seg_off[s];
        unsigned long long len = seg_len[s], off = 0;
        while (off < len) {
            unsigned char* data; unsigned long long datalen; int fin, type;
            int r = websocketframeDecode(p + off, len - off, &data, &datalen, &fin, &type);
            if (r <= 0) break;
            off += (unsigned int)r;
            ++nf;
        }
        total += off;
    }
    *frames = nf;
    return total;
}

/*
 * Reassembly baseline: the same loop, with each frame delivered the way the reactor's
 * stream hook does for a fragment packet type (src/component/net_channel_ex.c:110-157,
 * merge_packet :55-79, streamtransportctx{Cache,Merge}RecvPacket
 * src/datastruct/transport_ctx.c:179-201): a frame that is not FIN, or arrives while
 * fragments are cached, is copied into a malloc'd packet appended to the connection's
 * list; a FIN frame closes the message — one cached packet is delivered as is, several
 * are merged into one malloc'd buffer (a second copy) — and a FIN frame with nothing
 * cached is delivered in place. The application callback (on_recv) folds the message
 * length and first/last bytes into a checksum so no copy can be elided. Restated glue
 * (the reactor itself is not buildable standalone); the decode is the reference's.
 */
#include <stdlib.h>
#include <string.h>

typedef struct RefPkt { struct RefPkt* next; unsigned long long len; unsigned char body[]; } RefPkt;

static unsigned long long ref_on_recv(const unsigned char* p, unsigned long long n) {
    return n ? n * 131u + p[0] * 7u + p[n - 1] : 1u;
}

__attribute__((visibility("default")))
unsigned long long ref_reassemble_segments(unsigned char* buf, const unsigned long long* seg_off,
                                           const unsigned long long* seg_len, unsigned int nseg,
                                           unsigned long long* messages) {
    unsigned long long sum = 0, nm = 0;
    unsigned int s;
    for (s = 0; s < nseg; ++s) {
        unsigned char* p = buf + seg_off[s];
        unsigned long long len = seg_len[s], off = 0;
        RefPkt *head = NULL, *tail = NULL;
        while (off < len) {
            unsigned char* data; unsigned long long datalen; int fin, type;
            int r = websocketframeDecode(p + off, len - off, &data, &datalen, &fin, &type);
            if (r <= 0) break;
            off += (unsigned int)r;
            if (head || !fin) {
                RefPkt* k = (RefPkt*)malloc(sizeof(RefPkt) + datalen);
                if (!k) return 0;
                k->next = NULL;
                k->len = datalen;
                memmove(k->body, data, datalen);
                if (tail) tail->next = k; else head = k;
                tail = k;
                if (!fin) continue;
                if (head == tail) {
                    sum += ref_on_recv(head->body, head->len);
                    free(head);
                } else {
                    unsigned long long tot = 0, o = 0;
                    RefPkt *c, *n;
                    unsigned char* m;
                    for (c = head; c; c = c->next) tot += c->len;
                    m = (unsigned char*)malloc(tot ? tot : 1);
                    if (!m) return 0;
                    for (c = head; c; c = n) {
                        n = c->next;
                        memmove(m + o, c->body, c->len);
                        o += c->len;
                        free(c);
                    }
                    sum += ref_on_recv(m, tot);
                    free(m);
                }
                head = tail = NULL;
                ++nm;
            } else {
                sum += ref_on_recv(data, datalen);
                ++nm;
            }
        }
        while (head) { RefPkt* n = head->next; free(head); head = n; }   /* connection closed */
    }
    *messages = nm;
    return sum;
}

/*
 * Encode baseline (client side): every frame's header from the
 * reference's websocketframeEncodeHeadLength/websocketframeEncode
 * (src/crt/protocol/websocketframe.c:167-202), then — as a client must (RFC 6455 §5.3),
 * which the reference encoder leaves to its caller — the MASK bit, the 4 key bytes and
 * the payload copied with the same per-byte XOR loop the reference uses to unmask
 * (websocketframe.c:153-158). Frames are laid out back to back in dst. Returns bytes
 * written.
 */
unsigned int websocketframeEncodeHeadLength(unsigned long long datalen);
void websocketframeEncode(void* headbuf, int is_fin, int prev_is_fin, int type, unsigned long long datalen);

__attribute__((visibility("default")))
unsigned long long ref_encode_frames(const unsigned char* src, const unsigned long long* src_off,
                                     const unsigned long long* len, const unsigned int* key, unsigned int n,
                                     unsigned char* dst) {
    unsigned long long o = 0;
    unsigned int i;
    for (i = 0; i < n; ++i) {
        unsigned int hl = websocketframeEncodeHeadLength(len[i]);
        unsigned char* h = dst + o;
        const unsigned char* p = src + src_off[i];
        unsigned char* d;
        unsigned char k[4];
        unsigned long long j;
        websocketframeEncode(h, 1, 1, 2, len[i]);
        h[1] |= 0x80;
        k[0] = (unsigned char)key[i]; k[1] = (unsigned char)(key[i] >> 8);
        k[2] = (unsigned char)(key[i] >> 16); k[3] = (unsigned char)(key[i] >> 24);
        memcpy(h + hl, k, 4);
        d = h + hl + 4;
        for (j = 0; j < len[i]; ++j) d[j] = p[j] ^ k[j % 4];
        o += hl + 4 + len[i];
    }
    return o;
}

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

/*
 * ws_synth.h — seeded, counter-based synthetic WebSocket frame generator.
 *
 * Test/bench INPUT generator only (not the decode path). Header-only so the
 * same definition is compiled by gcc (host fill, CPU baseline, fixtures) and
 * by hipcc (on-device fill of multi-GiB batches): identical seed -> identical
 * bytes on both sides, so hashes and byte compares line up.
 *
 * Wire layout follows the reference encoder (websocketframe.c:167-202,
 * websocketframeEncodeHeadLength / websocketframeEncode): 2/4/10-byte header
 * by payload length (<126, <=0xFFFF, else), big-endian extended length
 * (memfunc.c:152-156,176-180). The reference encoder never sets MASK, so the
 * generator sets b1|=0x80 and appends the 4-byte key (RFC 6455 5.2/5.3),
 * exactly as a client would send it; payload byte i is plain[i]^key[i%4].
 *
 * Counter-based: every byte is a pure function of (seed, frame index, byte
 * index), so any thread can produce any byte independently.
 */
#ifndef UTIL_AMD_WS_SYNTH_H
#define UTIL_AMD_WS_SYNTH_H

#ifdef __HIPCC__
#define WS_HD __host__ __device__ __forceinline__
#else
#define WS_HD static inline
#endif

typedef unsigned long long ws_u64;

/* payload length rules */
enum { WS_PLEN_FIXED = 0, WS_PLEN_MIX3 = 1 };
/* first-byte rules */
enum { WS_B0_BINARY = 0, WS_B0_TEXT = 1, WS_B0_FRAG16 = 2 };

/* splitmix64 output function */
WS_HD ws_u64 ws_mix64(ws_u64 z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

WS_HD ws_u64 ws_synth_fseed(ws_u64 seed, ws_u64 f) {
    return ws_mix64(seed ^ (f * 0xD1B54A32D192ED03ULL));
}

/* little-endian 32-bit masking key of frame f (key byte k = (key >> 8k) & 0xFF) */
WS_HD unsigned int ws_synth_key(ws_u64 seed, ws_u64 f) {
    return (unsigned int)ws_mix64(ws_synth_fseed(seed, f) ^ 0x6B6579ULL);
}

/* 8 plaintext payload bytes [8j, 8j+8) of frame f, little-endian */
WS_HD ws_u64 ws_synth_plain_word(ws_u64 seed, ws_u64 f, ws_u64 j) {
    return ws_mix64(ws_synth_fseed(seed, f) + 0x9E3779B97F4A7C15ULL * (j + 1));
}

WS_HD unsigned char ws_synth_plain_byte(ws_u64 seed, ws_u64 f, ws_u64 i) {
    return (unsigned char)(ws_synth_plain_word(seed, f, i >> 3) >> (8 * (i & 7)));
}

WS_HD ws_u64 ws_synth_plen(int plen_kind, ws_u64 fixed_len, ws_u64 seed, ws_u64 f) {
    if (plen_kind == WS_PLEN_MIX3) {
        ws_u64 r = ws_mix64(ws_synth_fseed(seed, f) ^ 0x4C454EULL) % 3ULL;
        return r == 0 ? 125ULL : (r == 1 ? 1500ULL : 65536ULL);
    }
    return fixed_len;
}

WS_HD unsigned char ws_synth_b0(int b0_kind, ws_u64 f) {
    if (b0_kind == WS_B0_TEXT) return 0x81;          /* FIN | TEXT */
    if (b0_kind == WS_B0_FRAG16) {                   /* 16-fragment message, a4 */
        unsigned j = (unsigned)(f & 15ULL);
        return j == 0 ? 0x02 : (j == 15 ? 0x80 : 0x00);
    }
    return 0x82;                                     /* FIN | BINARY */
}

/* header bytes excluding the mask key: websocketframe.c:167-174 */
WS_HD unsigned int ws_synth_headlen(ws_u64 plen) {
    return plen < 126 ? 2u : (plen <= 0xFFFFULL ? 4u : 10u);
}

/* full wire length of a masked frame */
WS_HD ws_u64 ws_synth_wirelen(ws_u64 plen) {
    return (ws_u64)ws_synth_headlen(plen) + 4ULL + plen;
}

/* header + key bytes (<= 14) of frame f into h[]; returns their count */
WS_HD unsigned int ws_synth_header(unsigned char* h, unsigned char b0, ws_u64 plen,
                                   unsigned int key) {
    unsigned int n = ws_synth_headlen(plen), i;
    h[0] = b0;
    if (n == 2) {
        h[1] = (unsigned char)(0x80 | plen);
    } else if (n == 4) {
        h[1] = 0x80 | 126;
        h[2] = (unsigned char)(plen >> 8);
        h[3] = (unsigned char)plen;
    } else {
        h[1] = 0x80 | 127;
        for (i = 0; i < 8; ++i) h[2 + i] = (unsigned char)(plen >> (56 - 8 * i));
    }
    for (i = 0; i < 4; ++i) h[n + i] = (unsigned char)(key >> (8 * i));
    return n + 4;
}

/* masked wire byte i of frame f (i indexes the whole wire frame) */
WS_HD unsigned char ws_synth_wire_byte(ws_u64 seed, ws_u64 f, unsigned char b0, ws_u64 plen,
                                       ws_u64 i) {
    unsigned int key = ws_synth_key(seed, f);
    unsigned int hl = ws_synth_headlen(plen) + 4u;
    if (i < hl) {
        unsigned char h[14];
        ws_synth_header(h, b0, plen, key);
        return h[i];
    }
    i -= hl;
    return (unsigned char)(ws_synth_plain_byte(seed, f, i) ^ (unsigned char)(key >> (8 * (i & 3))));
}

#endif

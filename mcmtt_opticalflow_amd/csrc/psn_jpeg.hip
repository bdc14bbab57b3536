// JPEG frame ingest on the device (include/psn_jpeg.h): the libjpeg baseline
// decode behind cv::imread (psn_where/main.cpp:144), restated for gfx950.
//
//   host   markers -> quantisation tables (natural order), Huffman tables
//          (canonical maxcode/valoffset + a 9-bit lookahead table), component
//          geometry, restart-segment byte offsets (RSTn positions); one pinned
//          staging block [tables | segment offsets | entropy bytes] -> one H2D
//   K1     jpeg_entropy_kernel: one thread per restart segment decodes its MCUs
//          (jdhuff.c: fill with 0xFF00 unstuffing, a marker feeds zeros; DC
//          prediction reset per segment) into int16 coefficient blocks
//   K2     jpeg_idct_kernel: one thread per 8x8 block, dequantise + islow IDCT
//          (jidctint.c, 64-bit intermediates as libjpeg-turbo's JLONG) + the
//          post-IDCT range-limit table -> component planes (u8)
//   K3     jpeg_color_kernel: one thread per pixel: fancy upsampling (jdsample.c
//          h2v1 / h2v2, edges replicated at the downsampled size), YCbCr->RGB
//          (jdcolor.c, SCALEBITS 16), BGR out
// Bit-identical to oracle/jpeg_oracle.c, which is pinned to libjpeg-turbo.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "psn_jpeg.h"
#include "psn_lk.h"

namespace psn {
namespace {

constexpr int kJpegMaxComp = 3;

struct HuffDev {            // one Huffman table (jdhuff.c d_derived_tbl)
    int maxcode[18];        // largest code of length l, -1 if none; [17] sentinel
    int valoff[18];         // vals index = code + valoff[l]
    uint16_t fast[512];     // 9-bit lookahead: (len << 8) | value, 0 = longer code
    uint8_t vals[256];
};

struct Tables {             // device copy per frame
    uint16_t qt[4][64];     // natural order
    HuffDev dc[4], ac[4];
};

struct CompGeo {
    int h, v, tq, td, ta;   // sampling factors, table selectors
    int bw, bh;             // blocks across / down (plane = bw*8 x bh*8)
    int dw, dh;             // downsampled size (edges of the fancy upsampler)
    int blk0;               // first coefficient block
    int plane0;             // byte offset of the plane
};

struct JpegArgs {
    int W, H, nc, hmax, vmax, mcux, nmcu, ri, nseg, data_len;
    CompGeo c[kJpegMaxComp];
    const Tables *tab;
    const int *seg;          // byte offset of each segment's first entropy byte
    const uint8_t *data;     // entropy-coded bytes
    int16_t *coef;           // [blocks][64], natural order
    uint8_t *planes;
    uint8_t *out;
    int out_stride;
    int nblocks;
};

__constant__ int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// Bit reader of one segment (jdhuff.c fill_bit_buffer semantics).
struct BitReader {
    const uint8_t *p;
    int pos, end;
    unsigned long long buf;
    int n;
    bool marker;
    __device__ void fill() {
        while (n <= 56) {
            unsigned c = 0;
            if (!marker && pos < end) {
                c = p[pos];
                if (c == 0xFF) {
                    int q = pos + 1;
                    while (q < end && p[q] == 0xFF) q++;  // fill bytes
                    if (q < end && p[q] == 0) {
                        pos = q + 1;  // stuffed zero: a 0xFF data byte
                    } else {
                        marker = true;  // a marker: zeros from here on
                        c = 0;
                    }
                } else {
                    pos++;
                }
            }
            buf |= (unsigned long long)c << (56 - n);
            n += 8;
        }
    }
    __device__ unsigned peek(int k) {
        if (n < k) fill();
        return (unsigned)(buf >> (64 - k));
    }
    __device__ void skip(int k) {
        buf <<= k;
        n -= k;
    }
    __device__ int bits(int k) {
        if (k == 0) return 0;
        const unsigned v = peek(k);
        skip(k);
        return (int)v;
    }
    __device__ int decode(const HuffDev &h) {
        const unsigned look = peek(16);
        const unsigned f = h.fast[look >> 7];
        if (f) {
            skip((int)(f >> 8));
            return (int)(f & 255);
        }
        for (int l = 10; l <= 16; l++) {
            const int code = (int)(look >> (16 - l));
            if (code <= h.maxcode[l]) {
                skip(l);
                return h.vals[(code + h.valoff[l]) & 255];
            }
        }
        skip(16);  // corrupt data: libjpeg warns and yields 0
        return 0;
    }
};

__device__ __forceinline__ int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

__global__ __launch_bounds__(64) void jpeg_entropy_kernel(JpegArgs A) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= A.nseg) return;
    const Tables &T = *A.tab;
    BitReader br;
    br.p = A.data;
    br.pos = A.seg[s];
    br.end = s + 1 < A.nseg ? A.seg[s + 1] : A.data_len;
    br.buf = 0;
    br.n = 0;
    br.marker = false;
    const int m0 = A.ri ? s * A.ri : 0, m1 = A.ri ? min(m0 + A.ri, A.nmcu) : A.nmcu;
    int last_dc[kJpegMaxComp] = {0, 0, 0};
    for (int mcu = m0; mcu < m1; mcu++) {
        const int mx = mcu % A.mcux, my = mcu / A.mcux;
        for (int ci = 0; ci < A.nc; ci++) {
            const CompGeo &g = A.c[ci];
            const int bh = A.nc == 1 ? 1 : g.h, bv = A.nc == 1 ? 1 : g.v;
            for (int by = 0; by < bv; by++)
                for (int bx = 0; bx < bh; bx++) {
                    int16_t *blk = A.coef + (size_t)(g.blk0 + (my * bv + by) * g.bw + mx * bh + bx) * 64;
                    const int sz = br.decode(T.dc[g.td]);
                    const int diff = sz ? extend(br.bits(sz), sz) : 0;
                    last_dc[ci] += diff;
                    blk[0] = (int16_t)last_dc[ci];
                    for (int k = 1; k < 64; k++) {
                        const int rs = br.decode(T.ac[g.ta]);
                        const int r = rs >> 4, sv = rs & 15;
                        if (sv) {
                            k += r;
                            blk[kNatural[k]] = (int16_t)extend(br.bits(sv), sv);
                        } else {
                            if (r != 15) break;
                            k += 15;
                        }
                    }
                }
        }
    }
}

__device__ __forceinline__ long long desc(long long x, int n) { return (x + (1LL << (n - 1))) >> n; }
__device__ __forceinline__ uint8_t range_limit(long long v) {
    const int idx = (int)(v & 1023);
    return (uint8_t)(idx < 128 ? idx + 128 : idx < 512 ? 255 : idx < 896 ? 0 : idx - 896);
}

// jidctint.c: one 1-D pass over 8 values (even part: rotator sqrt(2)*c(-6);
// odd part per figure 8), shared by columns and rows.
__device__ __forceinline__ void idct8(const long long (&d)[8], long long (&o)[8]) {
    const long long z1 = (d[2] + d[6]) * 4433;
    const long long t2 = z1 + d[6] * -15137, t3 = z1 + d[2] * 6270;
    const long long t0 = (d[0] + d[4]) * 8192, t1 = (d[0] - d[4]) * 8192;
    const long long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    long long a0 = d[7], a1 = d[5], a2 = d[3], a3 = d[1];
    long long z1o = a0 + a3, z2 = a1 + a2, z3 = a0 + a2, z4 = a1 + a3;
    const long long z5 = (z3 + z4) * 9633;
    a0 *= 2446;
    a1 *= 16819;
    a2 *= 25172;
    a3 *= 12299;
    z1o *= -7373;
    z2 *= -20995;
    z3 = z3 * -16069 + z5;
    z4 = z4 * -3196 + z5;
    a0 += z1o + z3;
    a1 += z2 + z4;
    a2 += z2 + z3;
    a3 += z1o + z4;
    o[0] = t10 + a3;
    o[7] = t10 - a3;
    o[1] = t11 + a2;
    o[6] = t11 - a2;
    o[2] = t12 + a1;
    o[5] = t12 - a1;
    o[3] = t13 + a0;
    o[4] = t13 - a0;
}

__global__ __launch_bounds__(256) void jpeg_idct_kernel(JpegArgs A) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= A.nblocks) return;
    int ci = 0;
    while (ci + 1 < A.nc && b >= A.c[ci + 1].blk0) ci++;
    const CompGeo &g = A.c[ci];
    const int lb = b - g.blk0, bx = lb % g.bw, by = lb / g.bw;
    const uint16_t *q = A.tab->qt[g.tq];
    const int16_t *blk = A.coef + (size_t)b * 64;
    int ws[64];
    for (int c = 0; c < 8; c++) {  // pass 1: columns, scaled by 2^PASS1_BITS
        long long d[8], o[8];
        for (int r = 0; r < 8; r++) d[r] = (long long)blk[8 * r + c] * q[8 * r + c];
        idct8(d, o);
        for (int r = 0; r < 8; r++) ws[8 * r + c] = (int)desc(o[r], 13 - 2);
    }
    uint8_t *dst = A.planes + g.plane0 + (size_t)(by * 8) * (g.bw * 8) + bx * 8;
    for (int r = 0; r < 8; r++) {  // pass 2: rows, descaled by 8 and 2^PASS1_BITS
        long long d[8], o[8];
        for (int k = 0; k < 8; k++) d[k] = ws[8 * r + k];
        idct8(d, o);
        uint32_t lo = 0, hi = 0;
        for (int k = 0; k < 4; k++) {
            lo |= (uint32_t)range_limit(desc(o[k], 13 + 2 + 3)) << (8 * k);
            hi |= (uint32_t)range_limit(desc(o[k + 4], 13 + 2 + 3)) << (8 * k);
        }
        uint32_t *row = (uint32_t *)(dst + (size_t)r * (g.bw * 8));
        row[0] = lo;
        row[1] = hi;
    }
}

// One fancy-upsampled chroma sample at full-resolution (x, y).
__device__ __forceinline__ int chroma(const JpegArgs &A, const CompGeo &g, int x, int y) {
    const uint8_t *pl = A.planes + g.plane0;
    const int pw = g.bw * 8;
    const int sx = A.hmax / g.h, sy = A.vmax / g.v;
    if (sx == 1 && sy == 1) return pl[(size_t)y * pw + x];
    const int i = x >> 1;
    if (sy == 1) {  // h2v1_fancy_upsample
        const uint8_t *row = pl + (size_t)y * pw;
        const int cur = row[i];
        if (g.dw == 1) return cur;
        if ((x & 1) == 0) return i == 0 ? cur : (cur * 3 + row[i - 1] + 1) >> 2;
        return i == g.dw - 1 ? cur : (cur * 3 + row[i + 1] + 2) >> 2;
    }
    const int j = y >> 1;  // h2v2_fancy_upsample
    const int jn = (y & 1) ? min(j + 1, g.dh - 1) : max(j - 1, 0);
    const uint8_t *r0 = pl + (size_t)j * pw, *r1 = pl + (size_t)jn * pw;
    const int cs = r0[i] * 3 + r1[i];
    if (g.dw == 1) return (cs * 4 + ((x & 1) ? 7 : 8)) >> 4;
    if ((x & 1) == 0) return i == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + r0[i - 1] * 3 + r1[i - 1] + 8) >> 4;
    return i == g.dw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + r0[i + 1] * 3 + r1[i + 1] + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)min(max(v, 0), 255); }

__global__ __launch_bounds__(256) void jpeg_color_kernel(JpegArgs A) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= A.W) return;
    const CompGeo &gy = A.c[0];
    const int Y = A.planes[gy.plane0 + (size_t)y * (gy.bw * 8) + x];
    uint8_t *o = A.out + (size_t)y * A.out_stride + 3 * x;
    if (A.nc == 1) {
        o[0] = o[1] = o[2] = (uint8_t)Y;
        return;
    }
    const int cb = chroma(A, A.c[1], x, y) - 128, cr = chroma(A, A.c[2], x, y) - 128;
    // jdcolor.c build_ycc_rgb_table: FIX(1.402) 91881, FIX(1.772) 116130, FIX(0.71414) 46802, FIX(0.34414) 22554
    const int r = (91881 * cr + 32768) >> 16, b = (116130 * cb + 32768) >> 16;
    const int gsum = (-22554 * cb + 32768) + (-46802 * cr);
    o[0] = clamp255(Y + b);
    o[1] = clamp255(Y + (gsum >> 16));
    o[2] = clamp255(Y + r);
}

int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

// jdhuff.c jpeg_make_d_derived_tbl: false for a table libjpeg rejects with
// JERR_BAD_HUFF_TABLE -- more codes of a length than fit after the shorter ones
// (the canonical code would overflow its length; the all-ones code is not
// allowed), or a DC symbol above 15. Checked before any table entry is written.
bool build_huff(const uint8_t *bits, const uint8_t *vals, int nvals, bool dc, HuffDev &h) {
    for (int l = 1, code = 0; l <= 16; l++) {
        code += bits[l - 1];
        if (code >= (1 << l)) return false;
        code <<= 1;
    }
    if (dc)
        for (int i = 0; i < nvals; i++)
            if (vals[i] > 15) return false;
    memset(&h, 0, sizeof h);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        h.valoff[l] = k - code;
        const int n = bits[l - 1];
        for (int i = 0; i < n && l <= 9; i++) {  // lookahead entries of the codes of length <= 9
            const int c = code + i, span = 1 << (9 - l);
            for (int j = 0; j < span; j++) h.fast[(c << (9 - l)) | j] = (uint16_t)((l << 8) | vals[(k + i) & 255]);
        }
        code += n;
        k += n;
        h.maxcode[l] = n ? code - 1 : -1;
        code <<= 1;
    }
    h.maxcode[17] = 0x7fffffff;
    for (int i = 0; i < 256; i++) h.vals[i] = i < nvals ? vals[i] : 0;
    return true;
}

}  // namespace
}  // namespace psn

struct psn_jpeg_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    uint8_t *d_blob = nullptr, *h_blob = nullptr;  // [Tables | segment offsets | entropy bytes]
    size_t blob_cap = 0;
    int16_t *d_coef = nullptr;
    size_t coef_cap = 0;
    uint8_t *d_planes = nullptr;
    size_t planes_cap = 0;
    hipEvent_t blob_free = nullptr;  // the previous frame's kernels have read the staging blob
    bool blob_pending = false;
    uint8_t *d_out = nullptr;  // psn_jpeg_decode's device BGR buffer
    size_t out_cap = 0;
    std::string err;
};

namespace {

const int kNaturalHost[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                              12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                              35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                              58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int jerr(psn_jpeg_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        char b[256];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        c->err = b;
    }
    return code;
}

// A parsed frame: tables, geometry, entropy segments.
struct Parsed {
    psn::Tables tab;
    psn::JpegArgs a{};
    std::vector<int> seg;
    size_t ent0 = 0, ent1 = 0;  // entropy bytes [ent0, ent1) of the file
    // per Huffman slot (class tc, index th): 0 never defined, 1 valid, -1 the last
    // definition is one jpeg_make_d_derived_tbl rejects -- an error only for a table
    // the scan uses (libjpeg builds the derived tables of the scan's components)
    int hstate[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
};

int parse(const uint8_t *d, size_t n, Parsed &P, std::string &why) {
    memset(&P.tab, 0, sizeof P.tab);
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return why = "not a JPEG (no SOI)", PSN_LK_ERR_ARG;
    int ids[psn::kJpegMaxComp] = {0, 0, 0};
    bool sof = false;
    size_t p = 2;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) return why = "marker expected", PSN_LK_ERR_ARG;
        const int m = d[p + 1];
        if (m == 0xFF) {
            p++;
            continue;
        }
        const int len = psn::rd16(d + p + 2);
        if (len < 2 || p + 2 + (size_t)len > n) return why = "truncated segment", PSN_LK_ERR_ARG;
        const uint8_t *s = d + p + 4;
        const int sl = len - 2;
        if (m == 0xDB) {
            for (int o = 0; o < sl;) {
                const int pq = s[o] >> 4, tq = s[o] & 15;
                if (tq > 3 || o + 1 + (pq ? 128 : 64) > sl) return why = "bad DQT", PSN_LK_ERR_ARG;
                for (int i = 0; i < 64; i++)
                    P.tab.qt[tq][kNaturalHost[i]] = (uint16_t)(pq ? psn::rd16(s + o + 1 + 2 * i) : s[o + 1 + i]);
                o += 1 + (pq ? 128 : 64);
            }
        } else if (m == 0xC4) {
            for (int o = 0; o < sl;) {
                const int tc = s[o] >> 4, th = s[o] & 15;
                if (tc > 1 || th > 3 || o + 17 > sl) return why = "bad DHT", PSN_LK_ERR_ARG;
                int cnt = 0;
                for (int l = 0; l < 16; l++) cnt += s[o + 1 + l];
                if (cnt > 256 || o + 17 + cnt > sl) return why = "bad DHT", PSN_LK_ERR_ARG;
                P.hstate[tc][th] = psn::build_huff(s + o + 1, s + o + 17, cnt, tc == 0, tc ? P.tab.ac[th] : P.tab.dc[th]) ? 1 : -1;
                o += 17 + cnt;
            }
        } else if (m == 0xC0 || m == 0xC1) {
            if (sl < 6 || s[0] != 8) return why = "not 8-bit", PSN_LK_ERR_UNSUPPORTED;
            P.a.H = psn::rd16(s + 1);
            P.a.W = psn::rd16(s + 3);
            P.a.nc = s[5];
            if ((P.a.nc != 1 && P.a.nc != 3) || sl < 6 + 3 * P.a.nc || !P.a.W || !P.a.H)
                return why = "unsupported component count", PSN_LK_ERR_UNSUPPORTED;
            for (int c = 0; c < P.a.nc; c++) {
                ids[c] = s[6 + 3 * c];
                P.a.c[c].h = s[7 + 3 * c] >> 4;
                P.a.c[c].v = s[7 + 3 * c] & 15;
                P.a.c[c].tq = s[8 + 3 * c] & 3;
                if (P.a.c[c].h < 1 || P.a.c[c].h > 2 || P.a.c[c].v < 1 || P.a.c[c].v > 2)
                    return why = "unsupported sampling", PSN_LK_ERR_UNSUPPORTED;
            }
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return why = "not baseline sequential Huffman", PSN_LK_ERR_UNSUPPORTED;
        } else if (m == 0xDD) {
            P.a.ri = sl >= 2 ? psn::rd16(s) : 0;
        } else if (m == 0xDA) {
            if (!sof || sl < 1 || s[0] != P.a.nc) return why = "unsupported scan", PSN_LK_ERR_UNSUPPORTED;
            for (int i = 0; i < P.a.nc; i++)
                for (int c = 0; c < P.a.nc; c++)
                    if (ids[c] == s[1 + 2 * i]) {
                        P.a.c[c].td = (s[2 + 2 * i] >> 4) & 3;
                        P.a.c[c].ta = s[2 + 2 * i] & 3;
                    }
            // the scan's tables (jdhuff.c start_pass_huff_decoder -> jpeg_make_d_derived_tbl:
            // JERR_NO_HUFF_TABLE, JERR_BAD_HUFF_TABLE)
            for (int c = 0; c < P.a.nc; c++)
                for (int tc = 0; tc < 2; tc++) {
                    const int st = P.hstate[tc][tc ? P.a.c[c].ta : P.a.c[c].td];
                    if (st == 0) return why = "Huffman table not defined", PSN_LK_ERR_ARG;
                    if (st < 0) return why = "bad DHT (code lengths or DC symbols)", PSN_LK_ERR_ARG;
                }
            P.ent0 = p + 2 + (size_t)len;
            break;
        }
        p += 2 + (size_t)len;
    }
    if (!sof || !P.ent0) return why = "no frame / scan header", PSN_LK_ERR_ARG;
    psn::JpegArgs &a = P.a;
    a.hmax = a.vmax = 1;
    for (int c = 0; c < a.nc; c++) {
        a.hmax = std::max(a.hmax, a.c[c].h);
        a.vmax = std::max(a.vmax, a.c[c].v);
    }
    // 4:4:4, 4:2:2 (h2v1) and 4:2:0 (h2v2) chroma; 4:4:0 (luma 1x2: a vertical-only
    // upsample, h1v2) has no path in jpeg_color_kernel's chroma() and is refused
    if (a.nc == 3 && (a.c[0].h != a.hmax || a.c[0].v != a.vmax || a.c[1].h != 1 || a.c[1].v != 1 || a.c[2].h != 1 ||
                      a.c[2].v != 1 || (a.hmax == 1 && a.vmax == 2)))
        return why = "unsupported sampling", PSN_LK_ERR_UNSUPPORTED;
    const int mcux = (a.W + 8 * a.hmax - 1) / (8 * a.hmax), mcuy = (a.H + 8 * a.vmax - 1) / (8 * a.vmax);
    int blk = 0, plane = 0;
    for (int c = 0; c < a.nc; c++) {
        psn::CompGeo &g = a.c[c];
        g.bw = a.nc == 1 ? (a.W + 7) / 8 : mcux * g.h;
        g.bh = a.nc == 1 ? (a.H + 7) / 8 : mcuy * g.v;
        g.dw = (int)(((long long)a.W * g.h + a.hmax - 1) / a.hmax);
        g.dh = (int)(((long long)a.H * g.v + a.vmax - 1) / a.vmax);
        g.blk0 = blk;
        g.plane0 = plane;
        blk += g.bw * g.bh;
        plane += g.bw * g.bh * 64;
    }
    a.nblocks = blk;
    a.mcux = a.nc == 1 ? a.c[0].bw : mcux;
    a.nmcu = a.nc == 1 ? a.c[0].bw * a.c[0].bh : mcux * mcuy;
    // entropy data runs to EOI (or the end); restart segments start after each RSTn
    P.seg.assign(1, 0);
    size_t q = P.ent0;
    while (q + 1 < n) {
        if (d[q] == 0xFF && d[q + 1] != 0x00 && d[q + 1] != 0xFF) {
            const int mk = d[q + 1];
            if (mk >= 0xD0 && mk <= 0xD7) {
                if (a.ri) P.seg.push_back((int)(q + 2 - P.ent0));
                q += 2;
                continue;
            }
            break;  // EOI or another marker ends the scan
        }
        q++;
    }
    P.ent1 = q;
    const int want = a.ri ? (a.nmcu + a.ri - 1) / a.ri : 1;
    if ((int)P.seg.size() < want) return why = "missing restart markers", PSN_LK_ERR_ARG;
    P.seg.resize((size_t)want);
    a.nseg = want;
    a.data_len = (int)(P.ent1 - P.ent0);
    return PSN_LK_OK;
}

}  // namespace

extern "C" {

int psn_jpeg_info(const uint8_t *data, size_t len, int *w, int *h, int *comps) {
    if (!data || !w || !h) return PSN_LK_ERR_ARG;
    Parsed P;
    std::string why;
    const int rc = parse(data, len, P, why);
    if (rc) return rc;
    *w = P.a.W;
    *h = P.a.H;
    if (comps) *comps = P.a.nc;
    return PSN_LK_OK;
}

int psn_jpeg_create(int device, psn_jpeg_ctx **out) {
    if (!out) return PSN_LK_ERR_ARG;
    *out = nullptr;
    psn_jpeg_ctx *c = new (std::nothrow) psn_jpeg_ctx();
    if (!c) return PSN_LK_ERR_NOMEM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->blob_free, hipEventDisableTiming) != hipSuccess) {
        psn_jpeg_destroy(c);
        return PSN_LK_ERR_HIP;
    }
    c->stream = c->own;
    *out = c;
    return PSN_LK_OK;
}

void psn_jpeg_destroy(psn_jpeg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void *p : {(void *)c->d_blob, (void *)c->d_coef, (void *)c->d_planes, (void *)c->d_out})
        if (p) (void)hipFree(p);
    if (c->h_blob) (void)hipHostFree(c->h_blob);
    if (c->blob_free) (void)hipEventDestroy(c->blob_free);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

const char *psn_jpeg_last_error(psn_jpeg_ctx *c) { return c ? c->err.c_str() : "null context"; }

int psn_jpeg_set_stream(psn_jpeg_ctx *c, void *s) {
    if (!c) return PSN_LK_ERR_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    return PSN_LK_OK;
}

#define JCHK(c, e)                                                                                      \
    do {                                                                                                \
        hipError_t e_ = (e);                                                                            \
        if (e_ != hipSuccess) return jerr((c), PSN_LK_ERR_HIP, "%s: %s", #e, hipGetErrorString(e_));   \
    } while (0)

int psn_jpeg_decode_device(psn_jpeg_ctx *c, const uint8_t *data, size_t len, uint8_t *d_bgr, int stride) {
    if (!c || !data || !d_bgr) return PSN_LK_ERR_ARG;
    Parsed P;
    std::string why;
    int rc = parse(data, len, P, why);
    if (rc) return jerr(c, rc, "%s", why.c_str());
    psn::JpegArgs &a = P.a;
    if (stride < 3 * a.W) return jerr(c, PSN_LK_ERR_ARG, "stride %d < 3 * width %d", stride, a.W);
    JCHK(c, hipSetDevice(c->device));
    const size_t off_seg = (sizeof(psn::Tables) + 15) & ~(size_t)15;
    const size_t off_data = (off_seg + 4 * P.seg.size() + 15) & ~(size_t)15;
    const size_t blob = off_data + (size_t)a.data_len + 16;
    if (c->blob_pending) {  // the staging blob is reused: the previous frame's H2D must be done
        JCHK(c, hipEventSynchronize(c->blob_free));
        c->blob_pending = false;
    }
    if (c->blob_cap < blob) {
        JCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_blob) (void)hipFree(c->d_blob);
        if (c->h_blob) (void)hipHostFree(c->h_blob);
        c->d_blob = c->h_blob = nullptr;
        c->blob_cap = 0;
        const size_t cap = blob + blob / 2;
        JCHK(c, hipMalloc(&c->d_blob, cap));
        JCHK(c, hipHostMalloc(&c->h_blob, cap, hipHostMallocDefault));
        c->blob_cap = cap;
    }
    const size_t coef = (size_t)a.nblocks * 64 * sizeof(int16_t), planes = (size_t)a.nblocks * 64;
    if (c->coef_cap < coef || c->planes_cap < planes) {
        JCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_coef) (void)hipFree(c->d_coef);
        if (c->d_planes) (void)hipFree(c->d_planes);
        c->d_coef = nullptr;
        c->d_planes = nullptr;
        c->coef_cap = c->planes_cap = 0;
        JCHK(c, hipMalloc(&c->d_coef, coef));
        JCHK(c, hipMalloc(&c->d_planes, planes));
        c->coef_cap = coef;
        c->planes_cap = planes;
    }
    memcpy(c->h_blob, &P.tab, sizeof(psn::Tables));
    memcpy(c->h_blob + off_seg, P.seg.data(), 4 * P.seg.size());
    memcpy(c->h_blob + off_data, data + P.ent0, (size_t)a.data_len);
    JCHK(c, hipMemcpyAsync(c->d_blob, c->h_blob, blob, hipMemcpyHostToDevice, c->stream));
    JCHK(c, hipEventRecord(c->blob_free, c->stream));
    c->blob_pending = true;
    JCHK(c, hipMemsetAsync(c->d_coef, 0, coef, c->stream));
    a.tab = (const psn::Tables *)c->d_blob;
    a.seg = (const int *)(c->d_blob + off_seg);
    a.data = c->d_blob + off_data;
    a.coef = c->d_coef;
    a.planes = c->d_planes;
    a.out = d_bgr;
    a.out_stride = stride;
    hipLaunchKernelGGL(psn::jpeg_entropy_kernel, dim3((a.nseg + 63) / 64), dim3(64), 0, c->stream, a);
    JCHK(c, hipGetLastError());
    hipLaunchKernelGGL(psn::jpeg_idct_kernel, dim3((a.nblocks + 255) / 256), dim3(256), 0, c->stream, a);
    JCHK(c, hipGetLastError());
    hipLaunchKernelGGL(psn::jpeg_color_kernel, dim3((a.W + 255) / 256, a.H), dim3(256), 0, c->stream, a);
    JCHK(c, hipGetLastError());
    return PSN_LK_OK;
}

int psn_jpeg_decode(psn_jpeg_ctx *c, const uint8_t *data, size_t len, uint8_t *bgr, int stride) {
    if (!c || !data || !bgr) return PSN_LK_ERR_ARG;
    int w = 0, h = 0;
    int rc = psn_jpeg_info(data, len, &w, &h, nullptr);
    if (rc) return jerr(c, rc, "bad JPEG headers");
    if (stride < 3 * w) return jerr(c, PSN_LK_ERR_ARG, "stride %d < 3 * width %d", stride, w);
    JCHK(c, hipSetDevice(c->device));
    const size_t need = (size_t)w * 3 * h;
    if (c->out_cap < need) {
        JCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_out) (void)hipFree(c->d_out);
        c->d_out = nullptr;
        c->out_cap = 0;
        JCHK(c, hipMalloc(&c->d_out, need));
        c->out_cap = need;
    }
    rc = psn_jpeg_decode_device(c, data, len, c->d_out, 3 * w);
    if (rc) return rc;
    JCHK(c, hipMemcpy2DAsync(bgr, stride, c->d_out, 3 * (size_t)w, 3 * (size_t)w, h, hipMemcpyDeviceToHost, c->stream));
    JCHK(c, hipStreamSynchronize(c->stream));
    return PSN_LK_OK;
}

}  // extern "C"

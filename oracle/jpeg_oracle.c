/*
 * oracle/jpeg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the JPEG decode behind the reference's frame ingest
 * cv::imread(path, IMREAD_COLOR) (psn_where/main.cpp:144) as libjpeg's default
 * decompression does it for baseline sequential JPEG: Huffman entropy decode
 * with restart intervals (jdhuff.c), dequantisation and the accurate integer
 * inverse DCT jpeg_idct_islow (jidctint.c, CONST_BITS 13 / PASS1_BITS 2, the
 * post-IDCT range-limit table of jdmaster.c), "fancy" triangle-filter chroma
 * upsampling for h2v1 / h2v2 (jdsample.c, edge rows and columns replicated at
 * the downsampled size), and the fixed-point YCbCr->RGB tables of jdcolor.c
 * (SCALEBITS 16); output in OpenCV's BGR order.
 *
 * Pinning: the restatement is checked bit for bit against the libjpeg-turbo
 * decoder that PIL links in this container (tests/golden/jpeg_*.npz, made by
 * tests/golden/make_jpeg_golden.py). The reference links OpenCV 2.4.6, whose
 * bundled IJG libjpeg 8 decodes subsampled chroma with a scaled 16x16 IDCT
 * instead of the triangle filter: for 4:2:0 / 4:2:2 frames that decoder is not
 * present here and parity with it is unpinned; 4:4:4 and grayscale frames
 * decode the same in both.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lk_oracle.h"

static const int kZigzag[64 + 16] = {  /* jpeg_natural_order + overflow guard (jutils.c) */
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct {
    int bits[17];
    int vals[256];
    int nvals;
    /* decoding: maxcode[l], valptr[l], mincode[l] (jdhuff.c jpeg_make_d_derived_tbl) */
    long maxcode[18];
    int valoffset[18];
    int defined;
} Huff;

typedef struct {
    int id, h, v, tq, td, ta;
    int bw, bh;            /* blocks across / down (MCU-padded) */
    int dw, dh;            /* downsampled size: ceil(W * h / hmax) */
    uint8_t *plane;        /* bw*8 x bh*8 samples */
    int last_dc;
} Comp;

typedef struct {
    const uint8_t *p;
    size_t n, pos;
    uint32_t buf;
    int nbits;
    int hit_marker;
} Bits;

static void huff_build(Huff *h) {
    /* jpeg_make_d_derived_tbl: codes in order of length */
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        h->valoffset[l] = k - code;
        if (h->bits[l]) {
            code += h->bits[l];
            k += h->bits[l];
            h->maxcode[l] = code - 1;
        } else {
            h->maxcode[l] = -1;
        }
        code <<= 1;
    }
    h->maxcode[17] = 0x7fffffffL;  /* sentinel */
}

/* jdhuff.c fill_bit_buffer: bytes, 0xFF00 -> 0xFF, a marker stops the fill (zeros are fed) */
static int get_bit(Bits *b) {
    if (b->nbits == 0) {
        int c = 0;
        if (!b->hit_marker && b->pos < b->n) {
            c = b->p[b->pos];
            if (c == 0xFF) {
                size_t q = b->pos + 1;
                while (q < b->n && b->p[q] == 0xFF) q++;  /* fill bytes */
                if (q < b->n && b->p[q] == 0x00) {
                    b->pos = q + 1;
                    c = 0xFF;
                } else {
                    b->hit_marker = 1;  /* a marker: supply zeros */
                    c = 0;
                }
            } else {
                b->pos++;
            }
        }
        b->buf = (uint32_t)c;
        b->nbits = 8;
    }
    b->nbits--;
    return (int)((b->buf >> b->nbits) & 1);
}

static int get_bits(Bits *b, int n) {
    int v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | get_bit(b);
    return v;
}

static int huff_decode(Bits *b, const Huff *h) {
    long code = get_bit(b);
    int l = 1;
    while (code > h->maxcode[l]) {
        code = (code << 1) | get_bit(b);
        l++;
        if (l > 16) return 0;  /* corrupt data: libjpeg warns and returns 0 */
    }
    return h->vals[(int)(code + h->valoffset[l]) & 0xff];
}

static int extend(int v, int s) { return v < (1 << (s - 1)) ? v + (int)((~0u) << s) + 1 : v; }

/* jidctint.c jpeg_idct_islow, with the jdmaster.c post-IDCT range-limit table */
#define CONST_BITS 13
#define PASS1_BITS 2
#define DESC(x, n) (((x) + (1L << ((n)-1))) >> (n))
static uint8_t range_limit(long v) {
    const int idx = (int)(v & 1023);
    if (idx < 128) return (uint8_t)(idx + 128);
    if (idx < 512) return 255;
    if (idx < 896) return 0;
    return (uint8_t)(idx - 896);
}
static void idct_islow(const int *coef, const uint16_t *q, uint8_t *out, int stride) {
    long ws[64];
    for (int c = 0; c < 8; c++) {
        const long d0 = (long)coef[c] * q[c], d1 = (long)coef[8 + c] * q[8 + c], d2 = (long)coef[16 + c] * q[16 + c];
        const long d3 = (long)coef[24 + c] * q[24 + c], d4 = (long)coef[32 + c] * q[32 + c];
        const long d5 = (long)coef[40 + c] * q[40 + c], d6 = (long)coef[48 + c] * q[48 + c];
        const long d7 = (long)coef[56 + c] * q[56 + c];
        long z1 = (d2 + d6) * 4433;
        const long t2 = z1 + d6 * -15137, t3 = z1 + d2 * 6270;
        const long t0 = (d0 + d4) << CONST_BITS, t1 = (d0 - d4) << CONST_BITS;
        const long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        long o0 = d7, o1 = d5, o2 = d3, o3 = d1;
        long zz1 = o0 + o3, zz2 = o1 + o2, zz3 = o0 + o2, zz4 = o1 + o3;
        const long z5 = (zz3 + zz4) * 9633;
        o0 *= 2446;
        o1 *= 16819;
        o2 *= 25172;
        o3 *= 12299;
        zz1 *= -7373;
        zz2 *= -20995;
        zz3 *= -16069;
        zz4 *= -3196;
        zz3 += z5;
        zz4 += z5;
        o0 += zz1 + zz3;
        o1 += zz2 + zz4;
        o2 += zz2 + zz3;
        o3 += zz1 + zz4;
        ws[c] = DESC(t10 + o3, CONST_BITS - PASS1_BITS);
        ws[56 + c] = DESC(t10 - o3, CONST_BITS - PASS1_BITS);
        ws[8 + c] = DESC(t11 + o2, CONST_BITS - PASS1_BITS);
        ws[48 + c] = DESC(t11 - o2, CONST_BITS - PASS1_BITS);
        ws[16 + c] = DESC(t12 + o1, CONST_BITS - PASS1_BITS);
        ws[40 + c] = DESC(t12 - o1, CONST_BITS - PASS1_BITS);
        ws[24 + c] = DESC(t13 + o0, CONST_BITS - PASS1_BITS);
        ws[32 + c] = DESC(t13 - o0, CONST_BITS - PASS1_BITS);
    }
    for (int r = 0; r < 8; r++) {
        const long *w = ws + 8 * r;
        long z1 = (w[2] + w[6]) * 4433;
        const long t2 = z1 + w[6] * -15137, t3 = z1 + w[2] * 6270;
        const long t0 = (w[0] + w[4]) << CONST_BITS, t1 = (w[0] - w[4]) << CONST_BITS;
        const long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        long o0 = w[7], o1 = w[5], o2 = w[3], o3 = w[1];
        long zz1 = o0 + o3, zz2 = o1 + o2, zz3 = o0 + o2, zz4 = o1 + o3;
        const long z5 = (zz3 + zz4) * 9633;
        o0 *= 2446;
        o1 *= 16819;
        o2 *= 25172;
        o3 *= 12299;
        zz1 *= -7373;
        zz2 *= -20995;
        zz3 *= -16069;
        zz4 *= -3196;
        zz3 += z5;
        zz4 += z5;
        o0 += zz1 + zz3;
        o1 += zz2 + zz4;
        o2 += zz2 + zz3;
        o3 += zz1 + zz4;
        const int n = CONST_BITS + PASS1_BITS + 3;
        uint8_t *o = out + (long)r * stride;
        o[0] = range_limit(DESC(t10 + o3, n));
        o[7] = range_limit(DESC(t10 - o3, n));
        o[1] = range_limit(DESC(t11 + o2, n));
        o[6] = range_limit(DESC(t11 - o2, n));
        o[2] = range_limit(DESC(t12 + o1, n));
        o[5] = range_limit(DESC(t12 - o1, n));
        o[3] = range_limit(DESC(t13 + o0, n));
        o[4] = range_limit(DESC(t13 - o0, n));
    }
}

static int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

/* jdcolor.c build_ycc_rgb_table (SCALEBITS 16) */
#define SCALEBITS 16
#define ONE_HALF (1L << (SCALEBITS - 1))
#define FIX(x) ((long)((x) * (1L << SCALEBITS) + 0.5))
static long cr_r[256], cb_b[256], cr_g[256], cb_g[256];
static void color_tables(void) {
    for (int i = 0; i < 256; i++) {
        const long x = i - 128;
        cr_r[i] = (FIX(1.40200) * x + ONE_HALF) >> SCALEBITS;
        cb_b[i] = (FIX(1.77200) * x + ONE_HALF) >> SCALEBITS;
        cr_g[i] = -FIX(0.71414) * x;
        cb_g[i] = -FIX(0.34414) * x + ONE_HALF;
    }
}
static uint8_t clamp255(long v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* One chroma sample of the fancy-upsampled plane at full-resolution (x, y). */
static int upsample(const Comp *c, int hmax, int vmax, int x, int y) {
    const int sx = hmax / c->h, sy = vmax / c->v, pw = c->bw * 8;
    if (sx == 1 && sy == 1) return c->plane[(long)y * pw + x];
    if (sx == 2 && sy == 1) {  /* h2v1_fancy_upsample */
        const uint8_t *row = c->plane + (long)y * pw;
        const int i = x >> 1, dw = c->dw;
        const int cur = row[i];
        if (dw == 1) return cur;
        if ((x & 1) == 0) return i == 0 ? cur : (cur * 3 + row[i - 1] + 1) >> 2;
        return i == dw - 1 ? cur : (cur * 3 + row[i + 1] + 2) >> 2;
    }
    if (sx == 2 && sy == 2) {  /* h2v2_fancy_upsample: rows replicated at the downsampled height */
        const int i = x >> 1, j = y >> 1, dw = c->dw, dh = c->dh;
        const int jn = (y & 1) ? (j + 1 < dh ? j + 1 : dh - 1) : (j > 0 ? j - 1 : 0);
        const uint8_t *r0 = c->plane + (long)j * pw, *r1 = c->plane + (long)jn * pw;
        const int cs = r0[i] * 3 + r1[i];
        if (dw == 1) return (cs * 4 + ((x & 1) ? 7 : 8)) >> 4;
        if ((x & 1) == 0) {
            if (i == 0) return (cs * 4 + 8) >> 4;
            const int ls = r0[i - 1] * 3 + r1[i - 1];
            return (cs * 3 + ls + 8) >> 4;
        }
        if (i == dw - 1) return (cs * 4 + 7) >> 4;
        const int ns = r0[i + 1] * 3 + r1[i + 1];
        return (cs * 3 + ns + 7) >> 4;
    }
    return -1;  /* unsupported sampling */
}

int oracle_jpeg_info(const uint8_t *d, size_t n, int *w, int *h, int *ncomp) {
    size_t p = 2;
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return -1;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) return -1;
        const int m = d[p + 1];
        if (m == 0xFF) { p++; continue; }
        const int len = rd16(d + p + 2);
        if (m == 0xC0 || m == 0xC1) {
            *h = rd16(d + p + 5);
            *w = rd16(d + p + 7);
            *ncomp = d[p + 9];
            return 0;
        }
        p += 2 + (size_t)len;
    }
    return -1;
}

/* Full decode to BGR (or gray for 1-component files, replicated to BGR).
 * Returns 0, or < 0 on unsupported / corrupt streams. */
int oracle_jpeg_decode_bgr(const uint8_t *d, size_t n, uint8_t *out, int out_stride) {
    static int tables = 0;
    if (!tables) {
        color_tables();
        tables = 1;
    }
    uint16_t qt[4][64];
    Huff hdc[4], hac[4];
    memset(hdc, 0, sizeof hdc);
    memset(hac, 0, sizeof hac);
    Comp cp[4];
    memset(cp, 0, sizeof cp);
    int W = 0, H = 0, nc = 0, ri = 0, rc = -1;
    size_t p = 2;
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return -1;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) return -2;
        const int m = d[p + 1];
        if (m == 0xFF) { p++; continue; }
        const int len = rd16(d + p + 2);
        const uint8_t *s = d + p + 4;
        if (m == 0xDB) {  /* DQT */
            int o = 0;
            while (o < len - 2) {
                const int pq = s[o] >> 4, tq = s[o] & 15;
                o++;
                for (int i = 0; i < 64; i++) {
                    qt[tq & 3][kZigzag[i]] = (uint16_t)(pq ? rd16(s + o + 2 * i) : s[o + i]);
                }
                o += pq ? 128 : 64;
            }
        } else if (m == 0xC4) {  /* DHT */
            int o = 0;
            while (o < len - 2) {
                const int tc = s[o] >> 4, th = s[o] & 3;
                Huff *hh = tc ? &hac[th] : &hdc[th];
                int cnt = 0;
                hh->bits[0] = 0;
                for (int l = 1; l <= 16; l++) {
                    hh->bits[l] = s[o + l];
                    cnt += s[o + l];
                }
                if (cnt > 256) return -2;
                /* jpeg_make_d_derived_tbl's JERR_BAD_HUFF_TABLE (code overflow, DC symbol
                 * > 15) is raised when a scan uses the table: remember it (defined = -1) */
                int bad = 0;
                for (int l = 1, code = 0; l <= 16; l++) {
                    code += hh->bits[l];
                    if (code >= (1 << l)) bad = 1;
                    code <<= 1;
                }
                for (int i = 0; i < cnt; i++)
                    if (tc == 0 && s[o + 17 + i] > 15) bad = 1;
                for (int i = 0; i < cnt && i < 256; i++) hh->vals[i] = s[o + 17 + i];
                hh->nvals = cnt;
                hh->defined = bad ? -1 : 1;
                if (!bad) huff_build(hh);
                o += 17 + cnt;
            }
        } else if (m == 0xC0 || m == 0xC1) {  /* SOF0 / SOF1 (8-bit Huffman sequential) */
            if (s[0] != 8) return -3;
            H = rd16(s + 1);
            W = rd16(s + 3);
            nc = s[5];
            if (nc != 1 && nc != 3) return -3;
            for (int c = 0; c < nc; c++) {
                cp[c].id = s[6 + 3 * c];
                cp[c].h = s[7 + 3 * c] >> 4;
                cp[c].v = s[7 + 3 * c] & 15;
                cp[c].tq = s[8 + 3 * c] & 3;
            }
        } else if (m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
            return -3;  /* progressive / lossless / arithmetic: not the baseline path */
        } else if (m == 0xDD) {
            ri = rd16(s);
        } else if (m == 0xDA) {  /* SOS: one interleaved scan */
            const int ns = s[0];
            if (ns != nc) return -3;
            for (int i = 0; i < ns; i++) {
                const int id = s[1 + 2 * i];
                for (int c = 0; c < nc; c++)
                    if (cp[c].id == id) {
                        cp[c].td = s[2 + 2 * i] >> 4;
                        cp[c].ta = s[2 + 2 * i] & 15;
                    }
            }
            /* the scan's tables: JERR_NO_HUFF_TABLE / JERR_BAD_HUFF_TABLE */
            for (int c = 0; c < nc; c++)
                if (hdc[cp[c].td & 3].defined != 1 || hac[cp[c].ta & 3].defined != 1) return -2;
            p += 2 + (size_t)len;
            rc = 0;
            break;
        }
        p += 2 + (size_t)len;
    }
    if (rc || !W || !H) return -4;
    int hmax = 1, vmax = 1;
    for (int c = 0; c < nc; c++) {
        hmax = cp[c].h > hmax ? cp[c].h : hmax;
        vmax = cp[c].v > vmax ? cp[c].v : vmax;
    }
    const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
    for (int c = 0; c < nc; c++) {
        if (nc == 1) {  /* non-interleaved single component: MCU = one block */
            cp[c].bw = (W + 7) / 8;
            cp[c].bh = (H + 7) / 8;
        } else {
            cp[c].bw = mcux * cp[c].h;
            cp[c].bh = mcuy * cp[c].v;
        }
        cp[c].dw = (int)(((long)W * cp[c].h + hmax - 1) / hmax);
        cp[c].dh = (int)(((long)H * cp[c].v + vmax - 1) / vmax);
        cp[c].plane = (uint8_t *)calloc((size_t)cp[c].bw * 8 * cp[c].bh * 8, 1);
        if (!cp[c].plane) return -5;
    }
    Bits b = {d + p, n - p, 0, 0, 0, 0};
    const int nmcu = nc == 1 ? cp[0].bw * cp[0].bh : mcux * mcuy;
    const int mcw = nc == 1 ? cp[0].bw : mcux;
    int coef[64];
    for (int mcu = 0; mcu < nmcu; mcu++) {
        if (ri && mcu > 0 && mcu % ri == 0) {  /* restart: byte-align, consume RSTn, reset DC */
            b.nbits = 0;
            b.hit_marker = 0;
            while (b.pos + 1 < b.n && !(b.p[b.pos] == 0xFF && b.p[b.pos + 1] >= 0xD0 && b.p[b.pos + 1] <= 0xD7)) b.pos++;
            if (b.pos + 1 < b.n) b.pos += 2;
            for (int c = 0; c < nc; c++) cp[c].last_dc = 0;
        }
        const int mx = mcu % mcw, my = mcu / mcw;
        for (int c = 0; c < nc; c++) {
            const int bh = nc == 1 ? 1 : cp[c].h, bv = nc == 1 ? 1 : cp[c].v;
            for (int by = 0; by < bv; by++)
                for (int bx = 0; bx < bh; bx++) {
                    memset(coef, 0, sizeof coef);
                    int sz = huff_decode(&b, &hdc[cp[c].td]);
                    int diff = sz ? extend(get_bits(&b, sz), sz) : 0;
                    cp[c].last_dc += diff;
                    coef[0] = cp[c].last_dc;
                    for (int k = 1; k < 64; k++) {
                        const int rs = huff_decode(&b, &hac[cp[c].ta]);
                        const int r = rs >> 4, s2 = rs & 15;
                        if (s2) {
                            k += r;
                            const int v = extend(get_bits(&b, s2), s2);
                            coef[kZigzag[k]] = v;
                        } else {
                            if (r != 15) break;
                            k += 15;
                        }
                    }
                    const int X = (mx * bh + bx) * 8, Y = (my * bv + by) * 8, pw = cp[c].bw * 8;
                    idct_islow(coef, qt[cp[c].tq], cp[c].plane + (long)Y * pw + X, pw);
                }
        }
    }
    for (int y = 0; y < H; y++) {
        uint8_t *o = out + (long)y * out_stride;
        for (int x = 0; x < W; x++) {
            const int Y = cp[0].plane[(long)y * cp[0].bw * 8 + x];
            if (nc == 1) {
                o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = (uint8_t)Y;
                continue;
            }
            const int cb = upsample(&cp[1], hmax, vmax, x, y), cr = upsample(&cp[2], hmax, vmax, x, y);
            if (cb < 0 || cr < 0 || cp[0].h != hmax || cp[0].v != vmax) {
                rc = -3;
                goto done;
            }
            o[3 * x + 2] = clamp255(Y + cr_r[cr]);
            o[3 * x + 1] = clamp255(Y + ((cb_g[cb] + cr_g[cr]) >> SCALEBITS));
            o[3 * x] = clamp255(Y + cb_b[cb]);
        }
    }
done:
    for (int c = 0; c < nc; c++) free(cp[c].plane);
    return rc;
}

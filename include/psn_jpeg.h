/*
 * include/psn_jpeg.h -- JPEG frame ingest on the device (part of libpsn_lk.so).
 *
 * Replaces the step before the Tracker2D path: cv::imread(path, IMREAD_COLOR)
 * of every camera's frame (psn_where/main.cpp:133-151, :144), whose BGR output
 * CPSNWhere_Tracker2D::Run converts with cvtColor(BGR2GRAY)
 * (PSNWhere_Tracker2D.cpp:256-263). Baseline sequential JPEG (SOF0/SOF1,
 * 8-bit, Huffman), 1 or 3 components, 4:4:4 / 4:2:2 / 4:2:0, with or without
 * restart intervals, decoded as libjpeg's defaults do: Huffman (jdhuff.c),
 * jpeg_idct_islow (jidctint.c), fancy triangle upsampling (jdsample.c),
 * fixed-point YCbCr->RGB (jdcolor.c), stored in OpenCV's BGR order.
 *
 * Device work per frame: one thread per restart interval decodes the entropy
 * data into coefficient blocks (a stream without restart markers is one
 * interval, decoded by one thread), one thread per 8x8 block runs the IDCT,
 * one thread per pixel pair upsamples the chroma, converts colour and writes
 * BGR. Results are bit-identical to libjpeg-turbo's decoder (the one PIL links)
 * -- see oracle/jpeg_oracle.c for the pinning and for where OpenCV 2.4.6's
 * bundled libjpeg 8 differs (subsampled chroma).
 *
 * Plain C; returns 0 (PSN_LK_OK) or a negative PSN_LK_ERR_* code.
 */
#ifndef PSN_JPEG_H
#define PSN_JPEG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct psn_jpeg_ctx psn_jpeg_ctx;

/* Frame geometry from the headers (host only, no device work). */
int psn_jpeg_info(const uint8_t *data, size_t len, int *width, int *height, int *components);

/* A decoder with its device scratch (grown on demand) and HIP stream. */
int psn_jpeg_create(int device, psn_jpeg_ctx **out);
void psn_jpeg_destroy(psn_jpeg_ctx *ctx);
const char *psn_jpeg_last_error(psn_jpeg_ctx *ctx);
int psn_jpeg_set_stream(psn_jpeg_ctx *ctx, void *hip_stream);

/* Decode into device memory: d_bgr receives height rows of width*3 bytes,
 * `stride` bytes apart. Asynchronous on the decoder's stream; `data` is copied
 * before the call returns. */
int psn_jpeg_decode_device(psn_jpeg_ctx *ctx, const uint8_t *data, size_t len, uint8_t *d_bgr, int stride);
/* The same into host memory (synchronous). */
int psn_jpeg_decode(psn_jpeg_ctx *ctx, const uint8_t *data, size_t len, uint8_t *bgr, int stride);

#ifdef __cplusplus
}
#endif
#endif /* PSN_JPEG_H */

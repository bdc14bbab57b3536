// Batched online Savitzky-Golay smoother (include/psn_sgsmooth.h): one
// CPSNWhere_SGSmooth::Insert (psn_where/PSNWhere_SGSmooth.cpp:91-103,
// Smoothing :226-272, Filter :274-287) per series and coordinate, one thread
// per series, for thousands of tracked-point trajectories per frame.
//
// An Insert recomputes the smoothed positions from refreshPos on:
//   bypass  (window <= degree)        the new raw value;
//   entire  (window changed, length <= span): every position (begin rows of
//           Qbegin, the moving filter with Qmid, end rows of Qend);
//   update  (same window)             position length-1-hf (Qmid) and the last
//           hf positions (Qend).
// Every value read lies in the last `span` raw values, which is all the
// device keeps per series (ring, coordinate-major). Sums run in the
// reference's order in IEEE double (no FMA contraction: the Makefile builds
// with -ffp-contract=off), so results are bit-identical to the reference.
// Qsets come from a host restatement of CalculateQ (:133-224).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "psn_lk.h"
#include "psn_sgsmooth.h"

namespace psn {
namespace {

// One Qset per window size w (odd, 1..span): Qbegin[hf][w], Qmid[w], Qend[hf][w]
// packed at off[w] as Qbegin | Qmid | Qend.
struct SgArgs {
    const float *in;
    int in_stride, nseries, dims, span, degree;
    const uint8_t *active;
    int *refresh;
    double *out;
    double *hist;     // [span][dims][nseries]
    int *len, *qrows;  // [nseries]
    const double *q;  // packed Qsets
    int qoff[PSN_SG_MAX_SPAN + 1];
};

// CPSNWhere_SGSmooth::CalculateQ restated (same operation order): the reduced
// QR factor of the Vandermonde matrix by classical Gram-Schmidt, then
// Qbegin = Q(1:hf,:)*Q' and Qend = Q(hf+2:end,:)*Q'.
void calculate_q(int w, int degree, std::vector<double> &qb, std::vector<double> &qm, std::vector<double> &qe) {
    const int hf = (w - 1) / 2, cols = degree + 1;
    qm.assign((size_t)w, 1.0 / (double)w);
    std::vector<double> V((size_t)w * cols, 1.0), Q((size_t)w * cols, 0.0);
    for (int order = 1; order <= degree; order++)
        for (int t = -hf, pos = order; t <= hf; t++, pos += cols) V[(size_t)pos] = std::pow((double)t, (double)order);
    for (int c = 0; c < cols; c++) {
        std::vector<double> proj((size_t)c, 0.0);
        for (int r = 0; r < w; r++) {
            const int pos = r * cols + c;
            Q[(size_t)pos] = V[(size_t)pos];
            for (int p = 0; p < c; p++) proj[(size_t)p] += Q[(size_t)(r * cols + p)] * V[(size_t)pos];
        }
        double norm = 0.0;
        for (int r = 0; r < w; r++) {
            const int pos = r * cols + c;
            for (int p = 0; p < c; p++) Q[(size_t)pos] -= proj[(size_t)p] * Q[(size_t)(r * cols + p)];
            norm += Q[(size_t)pos] * Q[(size_t)pos];
        }
        norm = std::sqrt(norm);
        for (int r = 0; r < w; r++) Q[(size_t)(r * cols + c)] /= norm;
    }
    qb.assign((size_t)hf * w, 0.0);
    qe.assign((size_t)hf * w, 0.0);
    int front = 0, back = (hf + 1) * cols;
    for (int r = 0, pos = 0; r < hf; r++) {
        int pq = 0;
        for (int c = 0; c < w; c++, pos++)
            for (int e = 0; e < cols; e++, pq++) {
                qb[(size_t)pos] += Q[(size_t)pq] * Q[(size_t)(front + e)];
                qe[(size_t)pos] += Q[(size_t)pq] * Q[(size_t)(back + e)];
            }
        front += cols;
        back += cols;
    }
}

constexpr int kSgFastSpan = 16;  // windows up to this size run from registers

__global__ __launch_bounds__(256) void sg_insert_kernel(SgArgs A) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.nseries) return;
    if (A.active && !A.active[i]) {
        A.refresh[i] = -1;
        return;
    }
    const int S = A.span, D = A.dims, N = A.nseries;
    int L = A.len[i];
    double *__restrict__ h = A.hist + i;
    double *__restrict__ o = A.out + (size_t)i * S * D;
    auto at = [&](int pos, int d) -> double { return h[((size_t)(pos % S) * D + d) * N]; };
    for (int d = 0; d < D; d++) h[((size_t)(L % S) * D + d) * N] = (double)A.in[(size_t)i * A.in_stride + d];
    L++;
    A.len[i] = L;
    int w = min(S, L);
    w -= (w + 1) % 2;
    if (w <= A.degree) {  // bypass: the raw value
        A.refresh[i] = L - 1;
        for (int d = 0; d < D; d++) o[d] = (double)A.in[(size_t)i * A.in_stride + d];
        return;
    }
    const int hf = (w - 1) / 2;
    const double *qb = A.q + A.qoff[w], *qm = qb + hf * w, *qe = qm + w;
    if (A.qrows[i] == w && w <= kSgFastSpan) {
        // steady state: position L-1-hf by the filter and the last hf rows, from
        // the last w samples held in registers (x[j] = sample L-1-j; static
        // indices, every load in flight at once)
        A.refresh[i] = L - 1 - hf;
        for (int d = 0; d < D; d++) {
            double x[kSgFastSpan];
#pragma unroll
            for (int j = 0; j < kSgFastSpan; j++) x[j] = j < w ? at(L - 1 - j, d) : 0.0;
            double acc = 0.0;
#pragma unroll
            for (int c = 0; c < kSgFastSpan; c++)  // Filter: newest sample first
                if (c < w) acc += qm[c] * x[c];
            o[d] = acc;
            for (int p = 0; p < hf; p++) {  // end rows: samples L-w .. L-1 in order
                const double *qr = qe + p * w + w - 1;
                double e = 0.0;
#pragma unroll
                for (int j = kSgFastSpan - 1; j >= 0; j--)
                    if (j < w) e += qr[-j] * x[j];
                o[(1 + p) * D + d] = e;
            }
        }
        return;
    }
    int k = 0;  // output row
    int mid0, mid1;  // smoothed positions of the moving filter [mid0, mid1)
    if (A.qrows[i] != w) {  // entire update (L <= span: every value is in the ring)
        A.qrows[i] = w;
        A.refresh[i] = 0;
        for (int p = 0; p < hf; p++, k++)
            for (int d = 0; d < D; d++) {
                double acc = 0.0;
                for (int c = 0; c < w; c++) acc += qb[p * w + c] * at(c, d);
                o[k * D + d] = acc;
            }
        mid0 = hf;
        mid1 = L - hf;
    } else {
        mid0 = L - 1 - hf;
        mid1 = L - hf;
        A.refresh[i] = mid0;
    }
    for (int p = mid0; p < mid1; p++, k++) {  // Filter: newest sample first
        const int dp = p + hf;
        for (int d = 0; d < D; d++) {
            double acc = 0.0;
            for (int c = 0; c < w && dp - c >= 0; c++) acc += qm[c] * at(dp - c, d);
            o[k * D + d] = acc;
        }
    }
    for (int p = 0; p < hf; p++, k++)  // end rows over the last w samples
        for (int d = 0; d < D; d++) {
            double acc = 0.0;
            for (int c = 0; c < w; c++) acc += qe[p * w + c] * at(L - w + c, d);
            o[k * D + d] = acc;
        }
}

}  // namespace
}  // namespace psn

struct psn_sg {
    int device = 0, nseries = 0, dims = 0, span = 0, degree = 0;
    hipStream_t own = nullptr, stream = nullptr;
    double *d_hist = nullptr, *d_q = nullptr, *d_out = nullptr;
    int *d_len = nullptr, *d_qrows = nullptr, *d_refresh = nullptr;
    float *d_in = nullptr;
    uint8_t *d_active = nullptr;
    int qoff[PSN_SG_MAX_SPAN + 1] = {};
};

extern "C" {

int psn_sg_create(int device, int nseries, int dims, int span, int degree, psn_sg **out) {
    if (!out || nseries <= 0 || dims < 1 || dims > 4 || span < 1 || span > PSN_SG_MAX_SPAN || degree < 0)
        return PSN_LK_ERR_ARG;
    *out = nullptr;
    psn_sg *s = new (std::nothrow) psn_sg();
    if (!s) return PSN_LK_ERR_NOMEM;
    s->device = device;
    s->nseries = nseries;
    s->dims = dims;
    s->span = span;
    s->degree = degree;
    std::vector<double> q;
    for (int w = 1; w <= span; w += 2) {
        if (w <= degree) continue;
        std::vector<double> qb, qm, qe;
        psn::calculate_q(w, degree, qb, qm, qe);
        s->qoff[w] = (int)q.size();
        q.insert(q.end(), qb.begin(), qb.end());
        q.insert(q.end(), qm.begin(), qm.end());
        q.insert(q.end(), qe.begin(), qe.end());
    }
    bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&s->own, hipStreamNonBlocking) == hipSuccess;
    const size_t n = (size_t)nseries;
    ok = ok && hipMalloc(&s->d_hist, n * span * dims * sizeof(double)) == hipSuccess;
    ok = ok && hipMalloc(&s->d_q, std::max<size_t>(q.size(), 1) * sizeof(double)) == hipSuccess;
    ok = ok && hipMalloc(&s->d_len, n * sizeof(int)) == hipSuccess && hipMalloc(&s->d_qrows, n * sizeof(int)) == hipSuccess;
    ok = ok && (q.empty() || hipMemcpy(s->d_q, q.data(), q.size() * sizeof(double), hipMemcpyHostToDevice) == hipSuccess);
    if (!ok) {
        psn_sg_destroy(s);
        return PSN_LK_ERR_HIP;
    }
    s->stream = s->own;
    const int rc = psn_sg_reset(s);
    if (rc) {
        psn_sg_destroy(s);
        return rc;
    }
    *out = s;
    return PSN_LK_OK;
}

void psn_sg_destroy(psn_sg *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (void *p : {(void *)s->d_hist, (void *)s->d_q, (void *)s->d_out, (void *)s->d_len, (void *)s->d_qrows,
                    (void *)s->d_refresh, (void *)s->d_in, (void *)s->d_active})
        if (p) (void)hipFree(p);
    if (s->own) (void)hipStreamDestroy(s->own);
    delete s;
}

int psn_sg_reset(psn_sg *s) {
    if (!s) return PSN_LK_ERR_ARG;
    if (hipSetDevice(s->device) != hipSuccess) return PSN_LK_ERR_HIP;
    if (hipMemsetAsync(s->d_len, 0, (size_t)s->nseries * sizeof(int), s->stream) != hipSuccess ||
        hipMemsetAsync(s->d_qrows, 0, (size_t)s->nseries * sizeof(int), s->stream) != hipSuccess)
        return PSN_LK_ERR_HIP;
    return PSN_LK_OK;
}

int psn_sg_set_stream(psn_sg *s, void *stream) {
    if (!s) return PSN_LK_ERR_ARG;
    s->stream = stream ? (hipStream_t)stream : s->own;
    return PSN_LK_OK;
}

int psn_sg_insert_device(psn_sg *s, const float *d_in, int in_stride, const uint8_t *d_active, int *d_refresh,
                         double *d_out) {
    if (!s || !d_in || !d_refresh || !d_out || in_stride < s->dims) return PSN_LK_ERR_ARG;
    if (hipSetDevice(s->device) != hipSuccess) return PSN_LK_ERR_HIP;
    psn::SgArgs a{};
    a.in = d_in;
    a.in_stride = in_stride;
    a.nseries = s->nseries;
    a.dims = s->dims;
    a.span = s->span;
    a.degree = s->degree;
    a.active = d_active;
    a.refresh = d_refresh;
    a.out = d_out;
    a.hist = s->d_hist;
    a.len = s->d_len;
    a.qrows = s->d_qrows;
    a.q = s->d_q;
    std::memcpy(a.qoff, s->qoff, sizeof(a.qoff));
    hipLaunchKernelGGL(psn::sg_insert_kernel, dim3((s->nseries + 255) / 256), dim3(256), 0, s->stream, a);
    return hipGetLastError() == hipSuccess ? PSN_LK_OK : PSN_LK_ERR_HIP;
}

int psn_sg_insert(psn_sg *s, const float *in, int in_stride, const uint8_t *active, int *refresh, double *out) {
    if (!s || !in || !refresh || !out || in_stride < s->dims) return PSN_LK_ERR_ARG;
    if (hipSetDevice(s->device) != hipSuccess) return PSN_LK_ERR_HIP;
    const size_t n = (size_t)s->nseries;
    if (!s->d_in) {
        if (hipMalloc(&s->d_in, n * in_stride * sizeof(float)) != hipSuccess ||
            hipMalloc(&s->d_active, n) != hipSuccess || hipMalloc(&s->d_refresh, n * sizeof(int)) != hipSuccess ||
            hipMalloc(&s->d_out, n * s->span * s->dims * sizeof(double)) != hipSuccess)
            return PSN_LK_ERR_HIP;
    }
    // host rows -> device (in_stride may exceed dims: copy only what the kernel reads)
    std::vector<float> packed(n * s->dims);
    for (size_t i = 0; i < n; i++)
        for (int d = 0; d < s->dims; d++) packed[i * s->dims + d] = in[i * in_stride + d];
    if (hipMemcpyAsync(s->d_in, packed.data(), packed.size() * sizeof(float), hipMemcpyHostToDevice, s->stream) !=
        hipSuccess)
        return PSN_LK_ERR_HIP;
    if (active && hipMemcpyAsync(s->d_active, active, n, hipMemcpyHostToDevice, s->stream) != hipSuccess)
        return PSN_LK_ERR_HIP;
    int rc = psn_sg_insert_device(s, s->d_in, s->dims, active ? s->d_active : nullptr, s->d_refresh, s->d_out);
    if (rc) return rc;
    if (hipMemcpyAsync(refresh, s->d_refresh, n * sizeof(int), hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
        hipMemcpyAsync(out, s->d_out, n * s->span * s->dims * sizeof(double), hipMemcpyDeviceToHost, s->stream) !=
            hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess)
        return PSN_LK_ERR_HIP;
    return PSN_LK_OK;
}

int psn_sg_lengths(psn_sg *s, int *lengths) {
    if (!s || !lengths) return PSN_LK_ERR_ARG;
    if (hipSetDevice(s->device) != hipSuccess) return PSN_LK_ERR_HIP;
    if (hipMemcpyAsync(lengths, s->d_len, (size_t)s->nseries * sizeof(int), hipMemcpyDeviceToHost, s->stream) !=
            hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess)
        return PSN_LK_ERR_HIP;
    return PSN_LK_OK;
}

}  // extern "C"

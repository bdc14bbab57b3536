// C-ABI implementation of include/psn_lk.h (host side of libpsn_lk.so).
//
// One psn_lk_ctx per camera replaces what CPSNWhere_Tracker2D kept for
// OpenCV: the 4-slot gray ring (m_vecPtGrayFrameBuffer, PSNWhere_Tracker2D.h:187,
// allocated at PSNWhere_Tracker2D.cpp:258-261) -- here a device ring of full
// pyramids, built ONCE per frame -- and the two calcOpticalFlowPyrLK call sites
// (:776-782, :871-877), which rebuilt both pyramids and the Scharr planes on
// every call.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "psn_lk.h"
#include "psn_jpeg.h"
#include "psn_gridfast.h"
#include "psn_lk_kernels.h"

using psn::LevelDev;

struct psn_lk_ctx {
    int device = 0;
    int width = 0, height = 0;
    int user_slots = 0, nslots = 0;  // user ring + 2 scratch slots (one-shot API)
    int nlevels = 0;                 // max_level_cap + 1
    hipStream_t own_stream = nullptr, stream = nullptr;
    // ingest overlap: pyramid builds on their own stream, ordered against the
    // LK launches by per-slot events: ready after every build (waited for by
    // every launch that reads the slot, on whatever stream it runs), free after
    // the reads (one event per reading stream, all waited for by the next build
    // into the slot)
    // psn_lk_push_frame_async builds go round-robin to kIngestStreams streams:
    // consecutive cameras' builds run side by side once their uploads land
    static constexpr int kIngestStreams = 2;
    hipStream_t ingest_streams[kIngestStreams] = {};
    hipStream_t ingest_stream = nullptr;  // ingest_streams[0]
    int ingest_rr = 0;
    // psn_lk_push_frame_async: host uploads on their own stream (copy engine), so
    // the uploads of several frames run back to back while their builds wait on
    // the ingest stream (created at the highest priority: a build gates later
    // LK launches and must not wait behind them for compute-unit slots)
    // Consecutive uploads go round-robin to kCopyStreams copy streams: the cameras
    // of a frame-set upload in parallel on two DMA engines (one engine moves a
    // 1080p BGR frame in ~0.3 ms). Two, not four: after a device sync the first
    // upload on each further copy stream held the host ~7 ms (round-4 A/B over
    // 4/2/1/0 copy streams, tools/gpu_envab.sh: 2 had the best segment median).
    static constexpr int kCopyStreams = 2;
    hipStream_t copy_streams[kCopyStreams] = {};
    hipStream_t copy_stream = nullptr;  // copy_streams[0]
    int copy_rr = 0;
    std::vector<hipEvent_t> copy_done;
    int overlap = PSN_LK_OVERLAP_OFF;
    // PSN_LK_OVERLAP_FUSED: the last pushed build is deferred and run inside
    // the next LK launch that does not read its slot (tail workgroups)
    bool pend = false;
    int pend_slot = -1;
    psn::PyrBuildArgs pend_args{};
    unsigned *d_ctr = nullptr;  // [2] fused-build work counter + finished workgroups
    int fused_helpers = 0;      // FUSED_HELPERS variant: tile-only workgroups per fused launch
    psn::RingGeo ring{};        // slot/level geometry passed to the single-tile kernel
    std::vector<hipEvent_t> slot_ready;
    std::vector<char> ready_rec;
    // per slot: its build generation (slot_ready re-recorded), and per stream the
    // generation that stream has waited for already (no repeated waits)
    std::vector<unsigned> build_gen;
    std::vector<std::vector<std::pair<hipStream_t, unsigned>>> waited;
    // per slot: per stream the event of the last launch on it that read the slot;
    // one event per launch, shared by every slot it read (refcounted, pooled)
    struct SharedEv {
        hipEvent_t e = nullptr;
        int refs = 0;
    };
    std::vector<SharedEv *> ev_all, ev_free;
    std::vector<std::vector<std::pair<hipStream_t, SharedEv *>>> slot_free;
    // psn_lk_push_frame_async: per-slot staging buffer of the uploaded frame
    std::vector<uint8_t *> d_stage;
    std::vector<size_t> stage_cap;
    std::vector<int> used_slots;  // scratch of track_device_impl
    psn_jpeg_ctx *jpeg = nullptr;  // psn_lk_push_frame_jpeg's decoder (on the ingest stream)
    uint8_t *d_pyr = nullptr;
    LevelDev *d_slots = nullptr;
    std::vector<LevelDev> h_slots;  // [nslots][kMaxLevels]
    std::vector<char> filled;
    // staging
    uint8_t *d_src = nullptr;
    size_t d_src_cap = 0;
    float *d_prev = nullptr, *d_next = nullptr, *d_err = nullptr;
    uint8_t *d_status = nullptr;
    size_t d_pts_cap = 0;
    // kernel-variant overrides (psn_lk_debug_set_variant; tests and experiments only):
    // THREADS = workgroup size, GENERIC = always the tiled kernel
    int force_threads = 0;
    bool force_generic = false;
    bool onewave = true;  // ONEWAVE 0: multi-wave iterations in the single-tile kernel
#ifndef PSN_ST_OVL_DEFAULT
#define PSN_ST_OVL_DEFAULT 1
#endif
    bool st_ovl = PSN_ST_OVL_DEFAULT != 0;  // ST_OVL 0: every level's A phase in the single-tile prologue
    bool poison_lds = false;                 // POISON_LDS 1: LK launches fill their LDS with a pattern first
    bool box = true;      // BOX 0: box windows run the row-tiled kernel instead of lk_kernel_bx
    // TILED_LDS: LDS budget of a tiled-kernel workgroup (bytes); 76 KB keeps two
    // workgroups per CU (Tracker2D box windows: 64x64 backward, 64x160 forward at 1080p)
    int tiled_lds = 76 * 1024;
    int num_cus = 256;  // compute units of the device (launch shaping)
    // large-window kernel (lk_kernel_lg): LARGE forces it for every query;
    // lg_lds = LDS budget of one of its workgroups (row bands of the window)
    bool force_large = false;
    int lg_lds = 24 * 1024;
    bool lg_jr = true;  // LG_JR: J region of the iterations in LDS where it fits
    // its window-value slots in HBM, one buffer per stream (launches on one
    // stream run in order; launches on different streams may overlap)
    struct LgWs {
        hipStream_t s = nullptr;
        void *p = nullptr;
        size_t bytes = 0;
        hipEvent_t done = nullptr;  // recorded on s after each launch that used a slot buffer of s
    };
    std::vector<LgWs> lg_ws;
    std::vector<void *> lg_retired;  // outgrown slot buffers, freed at destroy (hipFree would wait for the device)
    unsigned long long *d_stamps = nullptr;  // diagnostic build only
    unsigned long long *d_samples = nullptr;  // psn_lk_debug_count_samples
    bool count_samples = false;
    // GridFAST scratch (per-cell keypoints of one launch) and host-call outputs
    uint32_t *d_gf_kp = nullptr;
    int *d_gf_cnt = nullptr;
    size_t gf_kp_cap = 0, gf_cnt_cap = 0;
    float *d_gf_xy = nullptr;
    int *d_gf_oc = nullptr, *d_gf_ot = nullptr;
    size_t gf_out_cap = 0;  // rois x cap floats pairs
    int gf_nroi_cap = 0;
    // timing: event ring, 2 events per timed call
    int tcap = 0;
    std::vector<hipEvent_t> ev_push, ev_track;
    std::vector<int> track_tag;            // per timed track call: the kernel it ran (psn_lk_timing_launches)
    long n_push = 0, n_track = 0;          // timed calls
    long calls_push = 0, calls_track = 0;  // all calls since enable_timing
    int every = 1;                         // time every `every`-th call of each kind
    std::string err;
};

static int set_err(psn_lk_ctx *c, int code, const char *fmt, ...);
static int launch_build(psn_lk_ctx *c, const psn::PyrBuildArgs &a, hipStream_t s, int slot);

// Run a deferred (fused-mode) build now, as its own launch on the LK stream.
static int flush_pending(psn_lk_ctx *c) {
    if (!c->pend) return PSN_LK_OK;
    c->pend = false;
    return launch_build(c, c->pend_args, c->stream, c->pend_slot);
}

static int set_err(psn_lk_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

// slot events only order streams of one device: a device-scope release suffices
static const unsigned kSlotEventFlags = hipEventDisableTiming | hipEventReleaseToDevice;

#define HIPCHK(c, expr)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return set_err((c), PSN_LK_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                               \
    } while (0)

extern "C" {

int psn_lk_abi_version(void) { return PSN_LK_ABI_VERSION; }

void psn_lk_default_params(psn_lk_params *p) {
    if (!p) return;
    p->win_w = 21;
    p->win_h = 21;
    p->max_level = 3;
    p->term_type = PSN_LK_TERM_COUNT | PSN_LK_TERM_EPS;
    p->max_count = 30;
    p->epsilon = 0.01;
    p->flags = 0;
    p->min_eig_threshold = 1e-4;
}

int psn_lk_window_supported(int w, int h) {
    return w > 0 && h > 0 && w <= PSN_LK_MAX_WIN_WIDTH && (long long)h * ((w + 3) / 4) < (long long)PSN_LK_MAX_WIN_QUADS;
}

int psn_lk_effective_max_level(int width, int height, int win_w, int win_h, int max_level) {
    if (width <= 0 || height <= 0 || max_level < 0) return PSN_LK_ERR_ARG;
    int sw = width, sh = height;
    for (int level = 0; level <= max_level; level++) {
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win_w || sh <= win_h) return level;
    }
    return max_level;
}

// SDMA engine set-up. ROCr creates an SDMA engine's queue on the first copy that
// engine runs: ~15 ms inside hsa_amd_memory_async_copy_on_engine, then ~0
// (tools/probes/probe_sdma_engines: 16 engines on MI355X, H2D 6 MB). The HIP
// runtime spreads async copies over the idle engines, so a frame upload that
// lands on an engine for the first time stalls its caller (the bench's first
// timed step after the device sync before the timed region: ~8 ms). Every
// engine runs one 4-KB copy each way here, once per process and device.
namespace {
struct AgentPick {
    uint32_t bdf = 0, domain = 0;
    char uuid[17] = {};  // the HIP device's UUID (16 characters), empty when HIP has none
    hsa_agent_t gpu{}, cpu{};
    int n_bdf = 0;  // GPU agents on the device's PCI function (> 1: a partitioned device)
    bool have_gpu = false, have_cpu = false, uuid_match = false;
};
hsa_status_t pick_agent(hsa_agent_t a, void *arg) {
    AgentPick *p = (AgentPick *)arg;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !p->have_cpu) {
        p->cpu = a;
        p->have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0, dom = 0;
        if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS ||
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) != HSA_STATUS_SUCCESS ||
            bdf != p->bdf || dom != p->domain)
            return HSA_STATUS_SUCCESS;
        p->n_bdf++;
        // the agent's UUID ("GPU-" + 16 characters) against the HIP device's: on a
        // partitioned device several agents share the PCI function
        char u[32] = {};
        const bool um = p->uuid[0] &&
                        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, u) == HSA_STATUS_SUCCESS &&
                        strncmp(u + 4, p->uuid, 16) == 0;
        if (!p->have_gpu || (um && !p->uuid_match)) {
            p->gpu = a;
            p->have_gpu = true;
            p->uuid_match = um;
        }
    }
    return HSA_STATUS_SUCCESS;
}
void warm_sdma_engines(int device) {
    // PSN_LK_SDMA_WARMUP=0: skipped (no create-time cost; the first upload per
    // engine then stalls once, as without the warm-up)
    const char *env = getenv("PSN_LK_SDMA_WARMUP");
    if (env && env[0] == '0') return;
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
        return;
    if (hsa_init() != HSA_STATUS_SUCCESS) return;  // reference-counted: the HIP runtime's instance
    AgentPick p;
    p.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
    p.domain = (uint32_t)dom;
    {
        hipUUID hu{};
        if (hipDeviceGetUuid(&hu, device) == hipSuccess) memcpy(p.uuid, hu.bytes, 16);
    }
    hsa_iterate_agents(pick_agent, &p);
    // several agents on the PCI function and none with the HIP device's UUID: the
    // engines of an unknown partition are not warmed (no stall fix, no harm)
    if (p.n_bdf > 1 && !p.uuid_match) p.have_gpu = false;
    void *h = nullptr, *d = nullptr;
    hsa_signal_t sig{};
    if (p.have_gpu && p.have_cpu && hipHostMalloc(&h, 4096, 0) == hipSuccess && hipMalloc(&d, 4096) == hipSuccess &&
        hsa_signal_create(1, 0, nullptr, &sig) == HSA_STATUS_SUCCESS) {
        for (int dir = 0; dir < 2; dir++) {
            const hsa_agent_t da = dir == 0 ? p.gpu : p.cpu, sa = dir == 0 ? p.cpu : p.gpu;
            void *dst = dir == 0 ? d : h;
            const void *src = dir == 0 ? h : d;
            uint32_t mask = 0;
            if (hsa_amd_memory_copy_engine_status(da, sa, &mask) != HSA_STATUS_SUCCESS) continue;
            for (int e = 0; e < 32; e++) {
                if (!(mask & (1u << e))) continue;
                hsa_signal_store_relaxed(sig, 1);
                if (hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, 4096, 0, nullptr, sig,
                                                        (hsa_amd_sdma_engine_id_t)(1u << e), true) == HSA_STATUS_SUCCESS)
                    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            }
        }
    }
    if (sig.handle) hsa_signal_destroy(sig);
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
    hsa_shut_down();
}
std::mutex g_warm_mu;
std::vector<std::pair<int, double>> g_warmed;  // devices whose engines are set up, with the wall ms it took
void warm_sdma_once(int device) {
    std::lock_guard<std::mutex> lk(g_warm_mu);
    for (const auto &w : g_warmed)
        if (w.first == device) return;
    const auto t0 = std::chrono::steady_clock::now();
    warm_sdma_engines(device);
    g_warmed.push_back({device, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count()});
}
}  // namespace

int psn_lk_sdma_warmup_ms(int device, double *ms) {
    if (!ms) return PSN_LK_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_warm_mu);
    for (const auto &w : g_warmed)
        if (w.first == device) {
            *ms = w.second;
            return PSN_LK_OK;
        }
    *ms = 0.0;
    return PSN_LK_ERR_ARG;  // no context was created on this device yet
}

int psn_lk_create(int device, int width, int height, int ring_slots, int max_level_cap, psn_lk_ctx **out) {
    if (!out || width <= 0 || height <= 0 || ring_slots <= 0 || max_level_cap < 0 ||
        max_level_cap > psn::kPyrMaxTop)
        return PSN_LK_ERR_ARG;
    // the pyramid tiles' LDS plan (guarded at build time for every top level:
    // psn::pyr_tiles_fit; kept here so a context never launches past the CU's LDS)
    if (psn::kStScratchBytes + psn::pyr_lds_bytes(max_level_cap, psn::pyr_tile_edge(max_level_cap)) > psn::kMaxLdsBytes)
        return PSN_LK_ERR_UNSUPPORTED;
    *out = nullptr;
    psn_lk_ctx *c = new (std::nothrow) psn_lk_ctx();
    if (!c) return PSN_LK_ERR_NOMEM;
    c->device = device;
    c->width = width;
    c->height = height;
    c->user_slots = ring_slots;
    c->nslots = ring_slots + 2;
    c->nlevels = max_level_cap + 1;
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->num_cus = cus;
    }
    auto fail = [&](int rc) {
        psn_lk_destroy(c);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    if (psn::lk_kernels_init() != hipSuccess) return fail(PSN_LK_ERR_HIP);
    warm_sdma_once(device);  // (before any stream work: the engines' queues exist from here on)
    if (hipMalloc(&c->d_ctr, 2 * sizeof(unsigned)) != hipSuccess) return fail(PSN_LK_ERR_NOMEM);
    if (hipMemset(c->d_ctr, 0, 2 * sizeof(unsigned)) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    c->stream = c->own_stream;
    {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return fail(PSN_LK_ERR_HIP);
        for (hipStream_t &is : c->ingest_streams)
            if (hipStreamCreateWithPriority(&is, hipStreamNonBlocking, greatest) != hipSuccess) return fail(PSN_LK_ERR_HIP);
        c->ingest_stream = c->ingest_streams[0];
        (void)least;
    }
    for (hipStream_t &cs : c->copy_streams)
        if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    c->copy_stream = c->copy_streams[0];
    // slot layout: levels back to back, rows padded to 256 B (one HBM burst / 4 x 64-B lines)
    size_t slot_bytes = 0;
    std::vector<size_t> lv_off(c->nlevels);
    std::vector<int> lw(c->nlevels), lh(c->nlevels), lp(c->nlevels);
    {
        int w = width, h = height;
        for (int l = 0; l < c->nlevels; l++) {
            lw[l] = w;
            lh[l] = h;
            lp[l] = (w + 255) & ~255;
            lv_off[l] = slot_bytes;
            slot_bytes += (size_t)lp[l] * h;
            w = (w + 1) / 2;
            h = (h + 1) / 2;
        }
    }
    slot_bytes = (slot_bytes + 4095) & ~(size_t)4095;
    // +256 B slack: the LK kernel's aligned dword staging loads may read up to
    // 3 bytes past the last row of a level
    if (hipMalloc(&c->d_pyr, slot_bytes * c->nslots + 256) != hipSuccess) return fail(PSN_LK_ERR_NOMEM);
    if (hipMemset(c->d_pyr, 0, slot_bytes * c->nslots + 256) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    c->ring.base = c->d_pyr;
    c->ring.slot_bytes = (long long)slot_bytes;
    for (int l = 0; l < c->nlevels; l++) {
        c->ring.off[l] = (long long)lv_off[l];
        c->ring.w[l] = lw[l];
        c->ring.h[l] = lh[l];
        c->ring.pitch[l] = lp[l];
    }
    c->h_slots.assign((size_t)c->nslots * psn::kMaxLevels, LevelDev{nullptr, 0, 0, 0, 0});
    for (int s = 0; s < c->nslots; s++)
        for (int l = 0; l < c->nlevels; l++)
            c->h_slots[(size_t)s * psn::kMaxLevels + l] = LevelDev{c->d_pyr + slot_bytes * s + lv_off[l], lw[l], lh[l], lp[l], 0};
    if (hipMalloc(&c->d_slots, sizeof(LevelDev) * c->h_slots.size()) != hipSuccess) return fail(PSN_LK_ERR_NOMEM);
    if (hipMemcpy(c->d_slots, c->h_slots.data(), sizeof(LevelDev) * c->h_slots.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(PSN_LK_ERR_HIP);
    c->filled.assign(c->nslots, 0);
    c->slot_ready.assign(c->nslots, nullptr);
    c->slot_free.assign(c->nslots, {});
    c->ready_rec.assign(c->nslots, 0);
    c->build_gen.assign(c->nslots, 0);
    c->waited.assign(c->nslots, {});
    c->d_stage.assign(c->nslots, nullptr);
    c->stage_cap.assign(c->nslots, 0);
    c->copy_done.assign(c->nslots, nullptr);
    for (int i = 0; i < c->nslots; i++) {
        if (hipEventCreateWithFlags(&c->slot_ready[i], kSlotEventFlags) != hipSuccess) return fail(PSN_LK_ERR_HIP);
        if (hipEventCreateWithFlags(&c->copy_done[i], kSlotEventFlags) != hipSuccess) return fail(PSN_LK_ERR_HIP);
    }
    *out = c;
    return PSN_LK_OK;
}

void psn_lk_destroy(psn_lk_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->pend && c->stream) (void)flush_pending(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    for (hipStream_t is : c->ingest_streams)
        if (is) (void)hipStreamSynchronize(is);
    for (hipStream_t cs : c->copy_streams)
        if (cs) (void)hipStreamSynchronize(cs);
    for (auto *v : {&c->ev_push, &c->ev_track, &c->slot_ready, &c->copy_done})
        for (auto e : *v)
            if (e) (void)hipEventDestroy(e);
    c->slot_free.clear();
    for (auto *se : c->ev_all) {
        (void)hipEventDestroy(se->e);
        delete se;
    }
    c->ev_all.clear();
    c->ev_free.clear();
    for (uint8_t *p : c->d_stage)
        if (p) (void)hipFree(p);
    if (c->jpeg) psn_jpeg_destroy(c->jpeg);
    // the last launch that used each stream's slot buffers (the current and the
    // retired ones: the stream runs in order) -- not the whole device, which
    // other contexts and groups share (a caller's stream may be gone by now, its
    // recorded event stays valid)
    for (auto &ws : c->lg_ws)
        if (ws.done) (void)hipEventSynchronize(ws.done);
    for (auto &ws : c->lg_ws) {
        if (ws.p) (void)hipFree(ws.p);
        if (ws.done) (void)hipEventDestroy(ws.done);
    }
    c->lg_ws.clear();
    for (void *p : c->lg_retired) (void)hipFree(p);
    c->lg_retired.clear();
    for (void *p : {(void *)c->d_samples, (void *)c->d_ctr, (void *)c->d_pyr, (void *)c->d_slots, (void *)c->d_src, (void *)c->d_prev, (void *)c->d_next,
                    (void *)c->d_err, (void *)c->d_status, (void *)c->d_gf_kp, (void *)c->d_gf_cnt, (void *)c->d_gf_xy,
                    (void *)c->d_gf_oc, (void *)c->d_gf_ot})
        if (p) (void)hipFree(p);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    for (hipStream_t is : c->ingest_streams)
        if (is) (void)hipStreamDestroy(is);
    for (hipStream_t cs : c->copy_streams)
        if (cs) (void)hipStreamDestroy(cs);
    delete c;
}

const char *psn_lk_last_error(psn_lk_ctx *c) { return c ? c->err.c_str() : "null context"; }

int psn_lk_set_stream(psn_lk_ctx *c, void *s) {
    if (!c) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);  // a deferred build belongs to the old stream's order
    if (rc) return rc;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return PSN_LK_OK;
}

void *psn_lk_get_stream(psn_lk_ctx *c) { return c ? (void *)c->stream : nullptr; }

int psn_lk_sync(psn_lk_ctx *c) {
    if (!c) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);
    if (rc) return rc;
    for (hipStream_t is : c->ingest_streams) HIPCHK(c, hipStreamSynchronize(is));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PSN_LK_OK;
}

int psn_lk_set_ingest_overlap(psn_lk_ctx *c, int mode) {
    if (!c || mode < PSN_LK_OVERLAP_OFF || mode > PSN_LK_OVERLAP_FUSED) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);
    if (rc) return rc;
    c->overlap = mode;
    return PSN_LK_OK;
}

int psn_lk_enable_timing(psn_lk_ctx *c, int capacity, int every) {
    if (!c || capacity < 0 || every < 1) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);
    if (rc) return rc;
    for (hipStream_t is : c->ingest_streams) HIPCHK(c, hipStreamSynchronize(is));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (auto *v : {&c->ev_push, &c->ev_track}) {
        for (auto e : *v)
            if (e) (void)hipEventDestroy(e);
        v->assign(2 * (size_t)capacity, nullptr);
        // timing-only events: no system-scope fence (cache writeback/invalidate) per record
        for (auto &e : *v) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    }
    c->tcap = capacity;
    c->track_tag.assign((size_t)capacity, 0);
    c->every = every;
    c->n_push = c->n_track = 0;
    c->calls_push = c->calls_track = 0;
    return PSN_LK_OK;
}

static int sum_events(psn_lk_ctx *c, std::vector<hipEvent_t> &ev, long n, double *ms) {
    *ms = 0.0;
    const long k = std::min<long>(n, c->tcap);
    for (long i = 0; i < k; i++) {
        HIPCHK(c, hipEventSynchronize(ev[2 * i + 1]));
        float t = 0.f;
        HIPCHK(c, hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
        *ms += t;
    }
    return PSN_LK_OK;
}

int psn_lk_timing_stats(psn_lk_ctx *c, int *n_push, double *push_ms, int *n_track, double *track_ms) {
    if (!c) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    double pm = 0, tm = 0;
    int rc = sum_events(c, c->ev_push, c->n_push, &pm);
    if (rc) return rc;
    rc = sum_events(c, c->ev_track, c->n_track, &tm);
    if (rc) return rc;
    if (n_push) *n_push = (int)std::min<long>(c->n_push, c->tcap);
    if (n_track) *n_track = (int)std::min<long>(c->n_track, c->tcap);
    if (push_ms) *push_ms = pm;
    if (track_ms) *track_ms = tm;
    c->n_push = c->n_track = 0;
    c->calls_push = c->calls_track = 0;
    return PSN_LK_OK;
}

int psn_lk_timing_launches(psn_lk_ctx *c, int cap, double *ms, int *tag, int *n) {
    if (!c || cap < 0 || !n || (cap > 0 && (!ms || !tag))) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const long k = std::min<long>(std::min<long>(c->n_track, c->tcap), cap);
    for (long i = 0; i < k; i++) {
        HIPCHK(c, hipEventSynchronize(c->ev_track[2 * i + 1]));
        float t = 0.f;
        HIPCHK(c, hipEventElapsedTime(&t, c->ev_track[2 * i], c->ev_track[2 * i + 1]));
        ms[i] = t;
        tag[i] = c->track_tag[(size_t)i];
    }
    *n = (int)k;
    return PSN_LK_OK;
}

int psn_lk_level_size(psn_lk_ctx *c, int level, int *w, int *h) {
    if (!c || level < 0 || level >= c->nlevels) return PSN_LK_ERR_ARG;
    if (w) *w = c->h_slots[level].w;
    if (h) *h = c->h_slots[level].h;
    return PSN_LK_OK;
}

// One standalone pyramid launch of `slot` on stream s (timed when timing is
// enabled); the slot's ready event is recorded after it.
static int launch_build(psn_lk_ctx *c, const psn::PyrBuildArgs &a, hipStream_t s, int slot) {
    const bool timed = c->tcap && (c->calls_push++ % c->every) == 0;
    const long ti = timed ? (c->n_push % c->tcap) : 0;
    if (timed) HIPCHK(c, hipEventRecord(c->ev_push[2 * ti], s));
    HIPCHK(c, psn::launch_pyramid(a, s));
    if (timed) {
        HIPCHK(c, hipEventRecord(c->ev_push[2 * ti + 1], s));
        c->n_push++;
    }
    HIPCHK(c, hipEventRecord(c->slot_ready[slot], s));
    c->ready_rec[slot] = 1;
    c->build_gen[slot]++;
    bool mine = false;  // the building stream is ordered after the build
    for (auto &w : c->waited[slot])
        if (w.first == s) w.second = c->build_gen[slot], mine = true;
    if (!mine) c->waited[slot].emplace_back(s, c->build_gen[slot]);
    return PSN_LK_OK;
}

// Make the current stream wait for the last build of `slot` (a no-op on the
// device when the build ran earlier on the same stream or has completed).
static int wait_slot_ready(psn_lk_ctx *c, int slot) {
    if (slot < 0 || slot >= c->nslots || !c->ready_rec[slot]) return PSN_LK_OK;
    // a stream that has waited for this build already is ordered after it
    for (auto &w : c->waited[slot])
        if (w.first == c->stream) {
            if (w.second == c->build_gen[slot]) return PSN_LK_OK;
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->slot_ready[slot], 0));
            w.second = c->build_gen[slot];
            return PSN_LK_OK;
        }
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->slot_ready[slot], 0));
    c->waited[slot].emplace_back(c->stream, c->build_gen[slot]);
    return PSN_LK_OK;
}

static void ev_unref(psn_lk_ctx *c, psn_lk_ctx::SharedEv *e) {
    if (e && --e->refs == 0) c->ev_free.push_back(e);
}

// After a launch on the current stream read `slots`: ONE event recorded behind
// it becomes that stream's free event of every slot read (a later build into
// one of them waits for it). An event returns to the pool when no slot refers
// to it; re-recording a pooled event never moves a live reference.
static int record_slots_free(psn_lk_ctx *c, const int *slots, int n) {
    psn_lk_ctx::SharedEv *e = nullptr;
    if (!c->ev_free.empty()) {
        e = c->ev_free.back();
        c->ev_free.pop_back();
    } else {
        e = new (std::nothrow) psn_lk_ctx::SharedEv();
        if (!e) return set_err(c, PSN_LK_ERR_NOMEM, "slot event");
        if (hipEventCreateWithFlags(&e->e, kSlotEventFlags) != hipSuccess) {
            delete e;
            return set_err(c, PSN_LK_ERR_HIP, "hipEventCreateWithFlags (slot event)");
        }
        c->ev_all.push_back(e);
    }
    HIPCHK(c, hipEventRecord(e->e, c->stream));
    for (int i = 0; i < n; i++) {
        const int slot = slots[i];
        if (slot < 0 || slot >= c->nslots) continue;
        bool found = false;
        for (auto &se : c->slot_free[slot])
            if (se.first == c->stream) {
                if (se.second != e) {
                    e->refs++;
                    ev_unref(c, se.second);
                    se.second = e;
                }
                found = true;
                break;
            }
        if (!found) {
            e->refs++;
            c->slot_free[slot].emplace_back(c->stream, e);
        }
    }
    if (e->refs == 0) c->ev_free.push_back(e);
    return PSN_LK_OK;
}

// Make stream s wait until every recorded read of `slot` is done (before a new build into it).
static int wait_slot_free(psn_lk_ctx *c, int slot, hipStream_t s) {
    for (auto &se : c->slot_free[slot])
        if (se.first != s) HIPCHK(c, hipStreamWaitEvent(s, se.second->e, 0));
    return PSN_LK_OK;
}

// Make stream s wait for the slot's last recorded build (it may run on another
// ingest stream and still read the slot's staging buffer or write its pyramid).
static int wait_prev_build(psn_lk_ctx *c, int slot, hipStream_t s) {
    if (c->ready_rec[slot]) HIPCHK(c, hipStreamWaitEvent(s, c->slot_ready[slot], 0));
    return PSN_LK_OK;
}

// Top-level tile of a standalone pyramid build (the level-0 region of a tile is
// 2^top * T + 3 * (2^top - 1) px square: larger tiles re-read less halo;
// psn::pyr_tile_edge, guarded against the LDS at build time).
// Pyramid-build arguments of `slot` from a device source frame.
static psn::PyrBuildArgs build_args(const psn_lk_ctx *c, int slot, const uint8_t *dev, int stride, int channels) {
    psn::PyrBuildArgs a{};
    a.src = dev;
    a.src_stride = stride;
    a.channels = channels;
    a.nlevels = c->nlevels;
    a.tile = psn::pyr_tile_edge(c->nlevels - 1);
    for (int l = 0; l < c->nlevels; l++) a.lv[l] = c->h_slots[(size_t)slot * psn::kMaxLevels + l];
    return a;
}

static int push_device_impl(psn_lk_ctx *c, int slot, const uint8_t *dev, int stride, int channels) {
    int rc = flush_pending(c);  // at most one deferred build
    if (rc) return rc;
    const psn::PyrBuildArgs a = build_args(c, slot, dev, stride, channels);
    c->filled[slot] = 1;
    if (c->overlap == PSN_LK_OVERLAP_FUSED && c->nlevels > 1) {
        c->ready_rec[slot] = 0;  // readers wait for the build by stream order (it runs first on the LK stream)
        c->pend = true;
        c->pend_slot = slot;
        c->pend_args = a;
        c->pend_args.tile = (c->nlevels - 1) <= 4 ? 8 : 4;  // inside the LK launch's LDS budget
        return PSN_LK_OK;
    }
    hipStream_t s = c->stream;
    if (c->overlap == PSN_LK_OVERLAP_STREAM) s = c->ingest_stream;  // once the slot's last readers are done
    rc = wait_slot_free(c, slot, s);
    if (rc) return rc;
    rc = wait_prev_build(c, slot, s);
    if (rc) return rc;
    return launch_build(c, a, s, slot);
}

// The slot's staging buffer, grown to `need` bytes (the old one may still be read by the ingest stream).
static int ensure_stage(psn_lk_ctx *c, int slot, size_t need) {
    if (c->stage_cap[slot] >= need) return PSN_LK_OK;
    for (hipStream_t cs : c->copy_streams) HIPCHK(c, hipStreamSynchronize(cs));
    for (hipStream_t is : c->ingest_streams) HIPCHK(c, hipStreamSynchronize(is));
    if (c->d_stage[slot]) (void)hipFree(c->d_stage[slot]);
    c->d_stage[slot] = nullptr;
    c->stage_cap[slot] = 0;
    HIPCHK(c, hipMalloc(&c->d_stage[slot], need));
    c->stage_cap[slot] = need;
    return PSN_LK_OK;
}

int psn_lk_push_frame_jpeg(psn_lk_ctx *c, int slot, const uint8_t *jpeg, size_t len) {
    if (!c || !jpeg) return PSN_LK_ERR_ARG;
    if (slot < 0 || slot >= c->user_slots) return set_err(c, PSN_LK_ERR_SLOT, "slot %d out of range", slot);
    int w = 0, h = 0;
    int rc = psn_jpeg_info(jpeg, len, &w, &h, nullptr);
    if (rc) return set_err(c, rc, "JPEG headers");
    if (w != c->width || h != c->height) return set_err(c, PSN_LK_ERR_ARG, "JPEG %dx%d, context %dx%d", w, h, c->width, c->height);
    HIPCHK(c, hipSetDevice(c->device));
    if ((rc = flush_pending(c))) return rc;
    if (!c->jpeg) {
        if ((rc = psn_jpeg_create(c->device, &c->jpeg))) return set_err(c, rc, "psn_jpeg_create");
        psn_jpeg_set_stream(c->jpeg, c->ingest_stream);
    }
    const size_t row = (size_t)c->width * 3;
    if ((rc = ensure_stage(c, slot, row * c->height))) return rc;
    if ((rc = wait_slot_free(c, slot, c->ingest_stream))) return rc;
    // the slot's previous build may still read d_stage[slot] (an async push builds
    // on either ingest stream): the decode overwrites it only after that build
    if ((rc = wait_prev_build(c, slot, c->ingest_stream))) return rc;
    rc = psn_jpeg_decode_device(c->jpeg, jpeg, len, c->d_stage[slot], (int)row);
    if (rc) return set_err(c, rc, "JPEG decode: %s", psn_jpeg_last_error(c->jpeg));
    c->filled[slot] = 1;
    return launch_build(c, build_args(c, slot, c->d_stage[slot], (int)row, 3), c->ingest_stream, slot);
}

int psn_lk_push_frame_async(psn_lk_ctx *c, int slot, const uint8_t *host, int stride, int channels) {
    if (!c || !host || (channels != 1 && channels != 3) || stride < c->width * channels) return PSN_LK_ERR_ARG;
    if (slot < 0 || slot >= c->user_slots) return set_err(c, PSN_LK_ERR_SLOT, "slot %d out of range", slot);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);
    if (rc) return rc;
    const size_t row = (size_t)c->width * channels, need = row * c->height;
    if ((rc = ensure_stage(c, slot, need))) return rc;
    hipStream_t s = c->ingest_streams[c->ingest_rr++ % psn_lk_ctx::kIngestStreams];
    hipStream_t cs = c->copy_streams[c->copy_rr++ % psn_lk_ctx::kCopyStreams];
    // the staging buffer is read only by this slot's previous build (its ready
    // event); the build waits for the upload and for every read of the slot
    if (c->ready_rec[slot]) HIPCHK(c, hipStreamWaitEvent(cs, c->slot_ready[slot], 0));
    if ((size_t)stride == row)  // contiguous rows: one linear copy (the DMA engine's fast path)
        HIPCHK(c, hipMemcpyAsync(c->d_stage[slot], host, need, hipMemcpyHostToDevice, cs));
    else
        HIPCHK(c, hipMemcpy2DAsync(c->d_stage[slot], row, host, stride, row, c->height, hipMemcpyHostToDevice, cs));
    HIPCHK(c, hipEventRecord(c->copy_done[slot], cs));
    rc = wait_slot_free(c, slot, s);
    if (rc) return rc;
    HIPCHK(c, hipStreamWaitEvent(s, c->copy_done[slot], 0));
    c->filled[slot] = 1;
    return launch_build(c, build_args(c, slot, c->d_stage[slot], (int)row, channels), s, slot);
}

int psn_lk_push_frame_device(psn_lk_ctx *c, int slot, const uint8_t *dev, int stride, int channels) {
    if (!c || !dev || (channels != 1 && channels != 3) || stride < c->width * channels) return PSN_LK_ERR_ARG;
    if (slot < 0 || slot >= c->user_slots) return set_err(c, PSN_LK_ERR_SLOT, "slot %d out of range", slot);
    HIPCHK(c, hipSetDevice(c->device));
    return push_device_impl(c, slot, dev, stride, channels);
}

static int push_host_impl(psn_lk_ctx *c, int slot, const uint8_t *host, int stride, int channels) {
    const size_t row = (size_t)c->width * channels, need = row * c->height;
    int rc0 = flush_pending(c);  // a deferred build may still read d_src's predecessor frame
    if (rc0) return rc0;
    if (c->d_src_cap < need) {
        if (c->d_src) (void)hipFree(c->d_src);
        c->d_src = nullptr;
        c->d_src_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_src, need));
        c->d_src_cap = need;
    }
    // the stream the build runs on (a fused-mode build of a host frame is not deferred)
    const int mode = c->overlap;
    if (mode == PSN_LK_OVERLAP_FUSED) c->overlap = PSN_LK_OVERLAP_OFF;
    hipStream_t s = c->overlap == PSN_LK_OVERLAP_STREAM ? c->ingest_stream : c->stream;
    hipError_t ce = hipMemcpy2DAsync(c->d_src, row, host, stride, row, c->height, hipMemcpyHostToDevice, s);
    int rc = ce == hipSuccess ? push_device_impl(c, slot, c->d_src, (int)row, channels)
                              : set_err(c, PSN_LK_ERR_HIP, "hipMemcpy2DAsync: %s", hipGetErrorString(ce));
    c->overlap = mode;
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(s));  // the host frame belongs to the caller after return
    return PSN_LK_OK;
}

int psn_lk_push_frame(psn_lk_ctx *c, int slot, const uint8_t *host, int stride, int channels) {
    if (!c || !host || (channels != 1 && channels != 3) || stride < c->width * channels) return PSN_LK_ERR_ARG;
    if (slot < 0 || slot >= c->user_slots) return set_err(c, PSN_LK_ERR_SLOT, "slot %d out of range", slot);
    HIPCHK(c, hipSetDevice(c->device));
    return push_host_impl(c, slot, host, stride, channels);
}

// Kernel classes of the planner: each track call's queries go to one launch per
// class (and per box-kernel build), each launch sized for its own windows.
enum LkClass { kClsSt = 0, kClsBx = 1, kClsTiled = 2, kClsLg = 3 };

// One query as planned: its device descriptor and the kernels that can take it.
struct PlannedQuery {
    int src = 0;  // index in the caller's query array
    psn::LkQueryDev d{};
    bool single = false;        // single-tile kernel (window <= 1024 px, LDS plan fits)
    int st_lds = 0;             // its LDS
    int ow_rows = 1 << 30, ow_lds = 0;  // its one-wave mode
    int ovl_lds = 0;                    // the one-wave mode with the overlapped A phase (0: does not fit)
    int bx_upt = 0, bx_lds = 0;  // box kernel units per thread (0: does not fit)
    int tiled_tr = 0;           // row-tiled kernel: tile rows (0: window not LDS-resident)
    int lg_tr = 0;              // large-window kernel: band rows
    bool lg_jr = false;         // + J region in LDS
    int lg_tq = 192;            // + quads per ordered-chain tile
    int cls = kClsLg, key = 0;  // the launch it goes to
};

// Row tiles of the row-tiled kernel (window LDS-resident): within the occupancy
// budget when the window allows, else the LDS limit; 0 if it does not fit.
static int tiled_rows(const psn_lk_ctx *c, int w, int h) {
    if ((long)w * h > 16384) return 0;  // Iw + Dw in LDS: 6 B per window pixel
    int tr = h;
    const int budget = 160 * 1024 - 1024;
    while (tr > 1 && psn::lk_lds_bytes(w, h, tr) > c->tiled_lds) tr--;
    while (tr > 1 && psn::lk_lds_bytes(w, h, tr) > budget) tr--;
    return psn::lk_lds_bytes(w, h, tr) <= budget ? tr : 0;
}
// Band rows of the large-window kernel's A phase within its LDS budget (>= 1 row;
// the tile planes of the fallbacks set the floor of the budget).
static int lg_rows(const psn_lk_ctx *c, int w, int h, bool jr, int tq) {
    int tr = 1;
    const int budget = std::max(c->lg_lds, psn::lg_lds_bytes(w, h, 1, jr, tq));
    while (tr < h && psn::lg_lds_bytes(w, h, tr + 1, jr, tq) <= budget) tr++;
    return tr;
}
// The large-window kernel's plan: the J region of the iterations in LDS with the
// largest ordered-chain tile (kLgTQs) that keeps the workgroup within
// kLgJrMaxLds (J staging needs the region's dword rows exactly divisible by the
// staging's magic: q * (d - 1) < 2^22 and q * magic < 2^32 for every dword q),
// else J from the level with kLgTQNoJr-quad tiles (measured with
// tools/gpu_lg_ab.sh, 512 points: 100x250 981 -> 858 us with 192-quad tiles;
// without the LDS J region 192-quad tiles were slower than 128 at 140x357).
static void lg_plan(const psn_lk_ctx *c, int w, int h, bool &jr, int &tq) {
    jr = false;
    tq = psn::kLgTQNoJr;
    if (!c->lg_jr) return;
    const long long d = psn::bx_jrp(w) / 4, n = (long long)psn::st_jreg_h(h) * d;
    if (!(n * (d - 1) < (1LL << 22) && n * (long long)psn::div_magic((int)d) < (1LL << 32))) return;
    for (int t : psn::kLgTQs)
        if (psn::lg_lds_bytes(w, h, 1, true, t) <= psn::kLgJrMaxLds) {
            jr = true;
            tq = t;
            return;
        }
}

// Validate and plan one query.
// no_bx16: a window of 13-16 units per thread goes to the large-window kernel
// (the call has large windows anyway: one launch fewer, see track_device_impl)
static int plan_query(psn_lk_ctx *c, const psn_lk_query &q, bool allow_scratch, PlannedQuery &pq,
                      bool no_bx16 = false) {
    const psn_lk_params &p = q.params;
    const int limit = allow_scratch ? c->nslots : c->user_slots;
    if (q.prev_slot < 0 || q.prev_slot >= limit || q.next_slot < 0 || q.next_slot >= limit)
        return set_err(c, PSN_LK_ERR_SLOT, "slot out of range (%d, %d)", q.prev_slot, q.next_slot);
    if (!c->filled[q.prev_slot] || !c->filled[q.next_slot])
        return set_err(c, PSN_LK_ERR_SLOT, "slot never filled (%d, %d)", q.prev_slot, q.next_slot);
    if (p.win_w <= 2 || p.win_h <= 2) return set_err(c, PSN_LK_ERR_WINSIZE, "winSize %dx%d <= 2", p.win_w, p.win_h);
    if (p.max_level < 0 || q.num_pts < 0 || q.first_pt < 0) return set_err(c, PSN_LK_ERR_ARG, "bad query");
    if (!psn_lk_window_supported(p.win_w, p.win_h))
        return set_err(c, PSN_LK_ERR_UNSUPPORTED, "window %dx%d wider than %d px or above 2^24 px", p.win_w, p.win_h,
                       PSN_LK_MAX_WIN_WIDTH);
    const int ml = psn_lk_effective_max_level(c->width, c->height, p.win_w, p.win_h, p.max_level);
    if (ml >= c->nlevels)
        return set_err(c, PSN_LK_ERR_LEVEL_CAP, "query needs %d levels, ring holds %d", ml + 1, c->nlevels);
    int max_count = (p.term_type & PSN_LK_TERM_COUNT) ? std::min(std::max(p.max_count, 0), 100) : 30;
    double eps = (p.term_type & PSN_LK_TERM_EPS) ? std::min(std::max(p.epsilon, 0.), 10.) : 0.01;
    const int w = p.win_w, h = p.win_h;
    const bool sse = (p.flags & PSN_LK_ACCUM_SCALAR) == 0;
    psn::LkQueryDev &d = pq.d;
    d = psn::LkQueryDev{};
    if ((long)w * h <= 256 * psn::kStEPTMax) {
        const psn::LkStLayout st(w, h, sse, ml + 1);
        if (st.total <= psn::kStMaxLds) {
            pq.single = true;
            pq.st_lds = st.total;
            const psn::LkStLayout so(w, h, sse, ml + 1, true);
            if (psn::ow_rows(w, h) <= psn::kOwMaxRows && so.total <= psn::kStMaxLds) {
                pq.ow_rows = psn::ow_rows(w, h);
                pq.ow_lds = so.total;
                const psn::LkStLayout sv(w, h, sse, ml + 1, true, true);
                if (sv.total <= psn::kStMaxLds) pq.ovl_lds = sv.total;
            }
        }
    }
    pq.tiled_tr = tiled_rows(c, w, h);
    lg_plan(c, w, h, pq.lg_jr, pq.lg_tq);
    pq.lg_tr = lg_rows(c, w, h, pq.lg_jr, pq.lg_tq);
    d.prev_slot = q.prev_slot;
    d.next_slot = q.next_slot;
    d.pt_begin = q.first_pt;
    d.num_pts = q.num_pts;
    d.win_w = w;
    d.win_h = h;
    d.max_level = ml;
    d.max_count = max_count;
    d.flags = p.flags;
    d.tile_rows = pq.single ? h : pq.tiled_tr;
    d.min_eig = (float)p.min_eig_threshold;
    d.eps2 = eps * eps;
    const int jrw = psn::st_jreg_w(w);
    const int nc = sse ? (w / 8) * 2 : 0;  // columns per SSE2 chain class
    d.ow_g = std::max(psn::ow_groups(w), 1);
    d.ow_rg = (h + d.ow_g - 1) / d.ow_g;
    d.dv_w = psn::div_magic(w);
    d.dv_dw = psn::div_magic(w + 1);
    d.dv_pm = psn::div_magic(psn::lk_pat_m(w));
    d.dv_jrw = psn::div_magic(jrw);
    d.dv_jrw4 = psn::div_magic(jrw / 4);
    d.dv_g = psn::div_magic(d.ow_g);
    d.dv_cw = psn::div_magic(nc);
    {  // box-window kernel: units of 4 pixels, <= kBxMaxUPT per thread
        const long need = ((long)h * psn::bx_qw(w) + psn::kBxNT - 1) / psn::kBxNT;
        const int upt = need <= 4 ? 4 : need <= 8 ? 8 : need <= 10 ? 10 : need <= 12 ? 12 : 16;
        const bool notail = sse && w % 8 == 0;
        // (a unit's J offset in the region, y * bx_jrp(w) + 4 q, is a 16-bit half)
        if (need <= psn::kBxMaxUPT && psn::BxLayout(w, h, upt).total <= psn::bx_max_lds(upt, notail) &&
            (long)psn::st_jreg_h(h) * psn::bx_jrp(w) < 65536) {
            pq.bx_upt = upt;
            pq.bx_lds = psn::BxLayout(w, h, upt).total;
            d.bx_tre = psn::bx_err_rows(w, h, psn::BxLayout(w, h, 4).pb);
            d.dv_bxpm = psn::div_magic(psn::bx_pm(w));
            d.dv_bxjr = psn::div_magic(psn::bx_jrp(w) / 4);
        }
    }
    // the class: the single-tile kernel for small windows, the box kernel for
    // Tracker2D boxes it holds in registers, else the large-window kernel (the
    // row-tiled kernel only when a variant asks for it and the window fits it)
    const bool forced = c->force_threads != 0;
    if (c->force_large) {
        pq.cls = kClsLg;
    } else if (pq.single && !c->force_generic) {
        pq.cls = kClsSt;
    } else if (pq.bx_upt > 0 && c->box && !c->force_generic && !forced && !(no_bx16 && pq.bx_upt == 16)) {
        pq.cls = kClsBx;
        pq.key = 10 * pq.bx_upt + ((sse && w % 8 == 0) ? 1 : 0);
    } else if (pq.tiled_tr > 0 && (c->force_generic || !c->box || forced)) {
        pq.cls = kClsTiled;
    } else {
        pq.cls = kClsLg;
    }
    if (pq.cls == kClsLg) {
        // (the kernel's LDS plan within the CU's: never an invalid launch)
        if (psn::lg_lds_bytes(w, h, pq.lg_tr, pq.lg_jr, pq.lg_tq) > psn::kMaxLdsBytes)
            return set_err(c, PSN_LK_ERR_UNSUPPORTED, "window %dx%d: large-window LDS plan above 160 KB", w, h);
        pq.key = pq.lg_tq;  // one launch per tile size
        d.tile_rows = pq.lg_tr;
        d.lg_jr = pq.lg_jr ? 1 : 0;
        if (pq.lg_jr) d.dv_bxjr = psn::div_magic(psn::bx_jrp(w) / 4);
    }
    if (pq.cls == kClsTiled) d.tile_rows = pq.tiled_tr;
    return PSN_LK_OK;
}

// The large-window kernel's slot buffer of the current stream, grown to `bytes`
// (to a power of two from 16 MB: the demand varies per call with the point
// count and window sizes). The outgrown buffer may still be read by launches in
// flight on the stream: it is retired, not freed, so growth never waits for
// the device (at most the geometric sum, < 2x the final size, stays reserved).
static int ensure_lg_ws(psn_lk_ctx *c, size_t bytes, void **out) {
    psn_lk_ctx::LgWs *ws = nullptr;
    for (auto &e : c->lg_ws)
        if (e.s == c->stream) ws = &e;
    if (!ws) {
        c->lg_ws.emplace_back();
        ws = &c->lg_ws.back();
        ws->s = c->stream;
    }
    if (ws->bytes < bytes) {
        size_t cap = (size_t)16 << 20;
        while (cap < bytes) cap <<= 1;
        void *p = nullptr;
        HIPCHK(c, hipMalloc(&p, cap));
        if (ws->p) c->lg_retired.push_back(ws->p);
        ws->p = p;
        ws->bytes = cap;
    }
    *out = ws->p;
    return PSN_LK_OK;
}
// HBM budget of one stream's large-window slots: one slot per point up to it,
// beyond it the grid strides (a slot per resident workgroup at the least)
static constexpr size_t kLgWsBudget = 512ull << 20;

// The launch just enqueued on c->stream built `slot` (a fused build): readers on
// other streams wait for that launch alone -- the event is recorded right after
// it, not after the call's later launches of other classes.
static int mark_fused_build(psn_lk_ctx *c, int slot) {
    HIPCHK(c, hipEventRecord(c->slot_ready[slot], c->stream));
    c->ready_rec[slot] = 1;
    c->build_gen[slot]++;
    bool mine = false;  // this stream built it: ordered after the build
    for (auto &w : c->waited[slot])
        if (w.first == c->stream) w.second = c->build_gen[slot], mine = true;
    if (!mine) c->waited[slot].emplace_back(c->stream, c->build_gen[slot]);
    return PSN_LK_OK;
}

// One launch of a planned group (queries of one class, <= kMaxQueries).
static int launch_group(psn_lk_ctx *c, std::vector<PlannedQuery *> &grp, int cls, int key, const float *d_prev,
                        float *d_next, uint8_t *d_status, float *d_err, const int *d_counts, int count_stride,
                        int &fused_slot) {
    psn::LkLaunchArgs a{};
    a.slots = c->d_slots;
    a.ring = c->ring;
    a.prev = d_prev;
    a.next = d_next;
    a.status = d_status;
    a.err = d_err;
    a.stamps = c->d_stamps;
    a.samples = c->count_samples ? c->d_samples : nullptr;
    a.counts = d_counts;
    a.count_stride = count_stride;
    int wgs = 0, maxpx = 0, rows_ow = 0, lds_ow = 0, lds = 0;
    for (size_t i = 0; i < grp.size(); i++) {
        PlannedQuery &pq = *grp[i];
        a.q[i] = pq.d;
        a.q[i].wg_begin = wgs;
        a.q[i].qidx = pq.src * count_stride;  // the query's count: d_counts[src * count_stride]
        wgs += pq.d.num_pts;
        maxpx = std::max(maxpx, pq.d.win_w * pq.d.win_h);
        rows_ow = std::max(rows_ow, pq.ow_rows);
        lds_ow = std::max(lds_ow, pq.ow_lds);
        lds = std::max(lds, pq.st_lds);
    }
    a.nq = (int)grp.size();
    if (wgs == 0) return PSN_LK_OK;
    const int forced = c->force_threads;
    if (cls == kClsSt) {
        // single-tile kernel: (workgroup size, window pixels per thread)
        int nt = maxpx <= 128 ? 64 : maxpx <= 256 ? 128 : 256;
        if (forced == 64 || forced == 128 || forced == 256 || forced == 512) {
            const int max_ept = forced == 512 ? 2 : psn::kStEPTMax;
            if (forced * max_ept >= maxpx) nt = forced;
        }
        const int ept = nt == 512 ? (maxpx <= 512 ? 1 : 2) : (maxpx <= 2 * nt ? 2 : 4);
        int threads = nt * 10 + ept;
        // one-wave iterations (wave 0 iterates, waves 1-3 stage the next level)
        if (c->onewave && !forced && rows_ow <= psn::kOwMaxRows) {
            const int oept = maxpx <= 512 ? 2 : 4;
            int E = rows_ow <= 4 ? 4 : rows_ow <= 7 ? 7 : rows_ow <= 8 ? 8 : 16;
            if (oept == 4 && E < 8) E = 8;
            threads = 1000 * E + 2560 + oept;
            lds = lds_ow;
            // more points than two workgroups per CU hold, and LDS for three:
            // the 168-VGPR variant (three per CU; one-camera launches fit at two)
            if (oept == 2 && E <= 8 && lds_ow <= 53 * 1024 && wgs > 2 * c->num_cus) {
                threads += 200000;
            } else if (c->st_ovl && E > 4) {
                // two workgroups per CU: the finer levels' A phase beside the
                // iterations, per query whose overlapped layout fits
                lds = 0;
                for (int i = 0; i < a.nq; i++) {
                    const PlannedQuery &pq = *grp[i];
                    a.q[i].st_ovl = pq.ovl_lds > 0 ? 1 : 0;
                    lds = std::max(lds, pq.ovl_lds > 0 ? pq.ovl_lds : pq.ow_lds);
                }
            }
        }
        bool builds = false;
        if (c->pend && fused_slot < 0 && !d_counts) {  // fuse the deferred build into this launch's tail
            int tx, ty, plds;
            psn::pyramid_grid(c->pend_args, tx, ty, plds);
            a.pyr = c->pend_args;
            a.pyr_ntiles = tx * ty;
            a.pyr_tiles_x = tx;
            a.pyr_ctr = c->d_ctr;
            // helpers start pulling tiles at once, so the build is done long before
            // the slowest points finish (tiles taken late would extend the launch)
            const int helpers = std::min(c->fused_helpers, a.pyr_ntiles);
            a.lk_wgs = wgs;
            a.total_wgs = wgs + helpers;
            wgs += helpers;
            lds = std::max(lds, psn::kStScratchBytes + plds);
            c->pend = false;
            fused_slot = c->pend_slot;
            builds = true;
        }
        a.poison_lds = c->poison_lds ? lds : 0;
        HIPCHK(c, psn::launch_lk(a, wgs, threads, lds, true, c->stream));
        return builds ? mark_fused_build(c, fused_slot) : PSN_LK_OK;
    }
    if (cls == kClsBx) {
        const int upt = key / 10;
        const bool notail = key % 10 != 0;
        // the launch's UPT sizes every query's fallback planes; tiles as large as the
        // kernel's occupancy (bx_occupancy) allows
        int lds_bx = 0;
        for (int i = 0; i < a.nq; i++) {
            psn::LkQueryDev &d = a.q[i];
            d.bx_hw = 1;
            while (d.bx_hw < 8 && psn::BxLayout(d.win_w, d.win_h, upt, d.bx_hw + 1).total <= psn::bx_lds_target(upt, notail))
                d.bx_hw++;
            lds_bx = std::max(lds_bx, psn::BxLayout(d.win_w, d.win_h, upt, d.bx_hw).total);
        }
        a.poison_lds = c->poison_lds ? lds_bx : 0;
        HIPCHK(c, psn::launch_lk_bx(a, wgs, upt, notail, lds_bx, c->stream));
        return PSN_LK_OK;
    }
    if (cls == kClsTiled) {
        int threads = maxpx <= 1024 ? 64 : maxpx <= 4096 ? 128 : 256;
        if (forced == 64 || forced == 128 || forced == 256) threads = forced;
        lds = 0;
        for (int i = 0; i < a.nq; i++) lds = std::max(lds, psn::lk_lds_bytes(a.q[i].win_w, a.q[i].win_h, a.q[i].tile_rows));
        HIPCHK(c, psn::launch_lk(a, wgs, threads, lds, false, c->stream));
        return PSN_LK_OK;
    }
    // large windows: one HBM slot per workgroup, the grid strides over the points
    long long slot = 0;
    lds = 0;
    for (int i = 0; i < a.nq; i++) {
        slot = std::max(slot, psn::lg_slot_int2(a.q[i].win_w, a.q[i].win_h));
        lds = std::max(lds, psn::lg_lds_bytes(a.q[i].win_w, a.q[i].win_h, a.q[i].tile_rows, a.q[i].lg_jr != 0, key));
    }
    const size_t slot_bytes = (size_t)slot * 8;
    // (within the budget also for the largest windows: one slot of a 2^24-px window
    // is ~100 MB, so no floor on the slot count past what the budget holds)
    const long long fit = std::max<long long>((long long)(kLgWsBudget / slot_bytes), 1);
    const int grid = (int)std::min<long long>(wgs, fit);
    void *ws = nullptr;
    int rc = ensure_lg_ws(c, slot_bytes * grid, &ws);
    if (rc) return rc;
    a.lg_ws = (int2 *)ws;
    a.lg_slot = slot;
    a.lk_wgs = wgs;
    a.total_wgs = wgs;
    a.poison_lds = c->poison_lds ? lds : 0;
    HIPCHK(c, psn::launch_lk_lg(a, grid, lds, key, c->stream));
    for (auto &e : c->lg_ws)
        if (e.s == c->stream) {
            if (!e.done) HIPCHK(c, hipEventCreateWithFlags(&e.done, hipEventDisableTiming));
            HIPCHK(c, hipEventRecord(e.done, c->stream));
        }
    return PSN_LK_OK;
}

static int kernel_tag(int cls, int key) { return cls == kClsBx ? key : cls == kClsSt ? 1 : cls == kClsTiled ? 2 : 3; }

static int track_device_impl(psn_lk_ctx *c, const psn_lk_query *q, int nq, const float *d_prev, float *d_next,
                             uint8_t *d_status, float *d_err, bool allow_scratch, const int *d_counts = nullptr,
                             int count_stride = 1) {
    if (d_counts && c->pend) {  // early-exit workgroups cannot take part in a fused build
        int rc = flush_pending(c);
        if (rc) return rc;
    }
    // plan every query first: a bad one fails the call before anything is launched
    std::vector<PlannedQuery> plan;
    plan.reserve((size_t)nq);
    for (int i = 0; i < nq; i++) {
        if (q[i].num_pts == 0) {
            if (q[i].params.win_w <= 2 || q[i].params.win_h <= 2)
                return set_err(c, PSN_LK_ERR_WINSIZE, "winSize %dx%d <= 2", q[i].params.win_w, q[i].params.win_h);
            continue;
        }
        plan.emplace_back();
        plan.back().src = i;
        int rc = plan_query(c, q[i], allow_scratch, plan.back());
        if (rc) return rc;
    }
    // The 16-unit box kernel (two workgroups per CU) beats the large-window kernel
    // on a launch of its own (512 points of 70x201: 513 vs 581 us), but a call
    // that holds large windows as well would launch one class more on the same
    // stream, each launch a fraction of the GPU with its own tail: there its
    // windows join the large-window launch (PETS-like boxes: 406 vs 450
    // camera-frames/s with the extra launch)
    if (std::any_of(plan.begin(), plan.end(), [](const PlannedQuery &pq) { return pq.cls == kClsLg; }))
        for (PlannedQuery &pq : plan)
            if (pq.cls == kClsBx && pq.bx_upt == 16) {
                PlannedQuery lq;
                lq.src = pq.src;
                int rc = plan_query(c, q[pq.src], allow_scratch, lq, true);
                if (rc) return rc;
                pq = lq;
            }
    // Consecutive caller queries with the same plan and the same point count,
    // their point blocks a constant stride apart, become one merged query of
    // sub-queries (LkQueryDev::sub_pts; each keeps its points, its device count
    // and its result slots, so the outputs are the same bits). Tracker2D's uniform
    // boxes are one query per camera then, not one per detection, and a call of
    // more than kMaxQueries detections -- configs[3]: 8 cameras x 32, the 4K Run:
    // 8 x 64 -- is one launch per kernel class instead of one per 32 detections,
    // each with its own tail.
    if (plan.size() > 1) {
        auto same_plan = [](const PlannedQuery &x, const PlannedQuery &y) {
            const psn::LkQueryDev &a = x.d, &b = y.d;
            return x.cls == y.cls && x.key == y.key && a.prev_slot == b.prev_slot && a.next_slot == b.next_slot &&
                   a.num_pts == b.num_pts && a.win_w == b.win_w && a.win_h == b.win_h &&
                   a.max_level == b.max_level && a.max_count == b.max_count && a.flags == b.flags &&
                   a.tile_rows == b.tile_rows && a.min_eig == b.min_eig && a.eps2 == b.eps2 && a.dv_w == b.dv_w &&
                   a.dv_dw == b.dv_dw && a.dv_pm == b.dv_pm && a.dv_jrw == b.dv_jrw && a.dv_jrw4 == b.dv_jrw4 &&
                   a.dv_g == b.dv_g && a.dv_cw == b.dv_cw && a.ow_g == b.ow_g && a.ow_rg == b.ow_rg &&
                   a.bx_tre == b.bx_tre && a.bx_hw == b.bx_hw && a.dv_bxpm == b.dv_bxpm && a.dv_bxjr == b.dv_bxjr &&
                   x.single == y.single && x.st_lds == y.st_lds && x.ow_rows == y.ow_rows && x.ow_lds == y.ow_lds &&
                   x.ovl_lds == y.ovl_lds && x.bx_upt == y.bx_upt && x.bx_lds == y.bx_lds &&
                   x.tiled_tr == y.tiled_tr && x.lg_tr == y.lg_tr && x.lg_jr == y.lg_jr && x.lg_tq == y.lg_tq;
        };
        size_t o = 0;
        int nsub = 1, stride = 0;  // sub-queries of plan[o] so far, their point stride
        for (size_t i = 1; i < plan.size(); i++) {
            const PlannedQuery &f = plan[o], &x = plan[i];
            const int sp = nsub == 1 ? x.d.pt_begin - f.d.pt_begin : stride;
            if (same_plan(f, x) && x.src == f.src + nsub && sp >= f.d.num_pts && sp > 0 &&
                x.d.pt_begin == f.d.pt_begin + nsub * sp) {
                stride = sp;
                nsub++;
                continue;
            }
            if (nsub > 1) {
                plan[o].d.sub_pts = plan[o].d.num_pts;
                plan[o].d.sub_pstride = stride;
                plan[o].d.num_pts *= nsub;
            }
            plan[++o] = plan[i];
            nsub = 1;
            stride = 0;
        }
        if (nsub > 1) {
            plan[o].d.sub_pts = plan[o].d.num_pts;
            plan[o].d.sub_pstride = stride;
            plan[o].d.num_pts *= nsub;
        }
        plan.resize(o + 1);
    }
    // slots built on the ingest stream must be complete before the LK reads them;
    // a deferred build of a slot this call reads runs first, as its own launch
    std::vector<int> &used = c->used_slots;  // distinct slots this call reads
    used.clear();
    for (const PlannedQuery &pq : plan)
        for (int sl : {pq.d.prev_slot, pq.d.next_slot})
            if (std::find(used.begin(), used.end(), sl) == used.end()) used.push_back(sl);
    for (int sl : used) {
        if (c->pend && sl == c->pend_slot) {
            int rc = flush_pending(c);
            if (rc) return rc;
        }
        int rc = wait_slot_ready(c, sl);
        if (rc) return rc;
    }
    // launch groups: (class, key) in a fixed order, queries in call order
    std::vector<std::pair<int, int>> groups;
    std::vector<long long> group_px;
    for (const PlannedQuery &pq : plan) {
        const std::pair<int, int> g(pq.cls, pq.key);
        const long long px = (long long)pq.d.win_w * pq.d.win_h * pq.d.num_pts;
        auto it = std::find(groups.begin(), groups.end(), g);
        if (it == groups.end()) {
            groups.push_back(g);
            group_px.push_back(px);
        } else {
            group_px[it - groups.begin()] += px;
        }
    }
    const bool timed = c->tcap && (c->calls_track++ % c->every) == 0;
    const long ti = timed ? (c->n_track % c->tcap) : 0;
    if (timed) HIPCHK(c, hipEventRecord(c->ev_track[2 * ti], c->stream));
    int fused_slot = -1;
    int launches = 0;
    std::vector<PlannedQuery *> grp;
    for (const auto &g : groups) {
        grp.clear();
        for (PlannedQuery &pq : plan) {
            if (pq.cls != g.first || pq.key != g.second) continue;
            grp.push_back(&pq);
            if ((int)grp.size() == psn::kMaxQueries) {
                int rc = launch_group(c, grp, g.first, g.second, d_prev, d_next, d_status, d_err, d_counts, count_stride,
                                      fused_slot);
                if (rc) return rc;
                launches++;
                grp.clear();
            }
        }
        if (!grp.empty()) {
            int rc = launch_group(c, grp, g.first, g.second, d_prev, d_next, d_status, d_err, d_counts, count_stride,
                                  fused_slot);
            if (rc) return rc;
            launches++;
        }
    }
    if (timed && !groups.empty()) {
        const size_t dom = (size_t)(std::max_element(group_px.begin(), group_px.end()) - group_px.begin());
        c->track_tag[(size_t)ti] = kernel_tag(groups[dom].first, groups[dom].second) + (groups.size() > 1 ? 1000 : 0);
    }
    if (c->pend) {  // no launch took it (no single-tile launch)
        int rc = flush_pending(c);
        if (rc) return rc;
    }
    if (timed) {
        HIPCHK(c, hipEventRecord(c->ev_track[2 * ti + 1], c->stream));
        c->n_track++;
    }
    (void)launches;
    // the next build into these slots waits for this launch
    if (!used.empty()) {
        int rc = record_slots_free(c, used.data(), (int)used.size());
        if (rc) return rc;
    }
    return PSN_LK_OK;
}

int psn_lk_track_device_counted(psn_lk_ctx *c, const psn_lk_query *q, int nq, const int *d_counts,
                                const float *d_prev, float *d_next, uint8_t *d_status, float *d_err) {
    return psn_lk_track_device_counted_strided(c, q, nq, d_counts, 1, d_prev, d_next, d_status, d_err);
}

int psn_lk_track_device_counted_strided(psn_lk_ctx *c, const psn_lk_query *q, int nq, const int *d_counts,
                                        int count_stride, const float *d_prev, float *d_next, uint8_t *d_status,
                                        float *d_err) {
    if (!c || !d_counts || count_stride < 1 || (nq > 0 && (!q || !d_prev || !d_next || !d_status)) || nq < 0)
        return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return track_device_impl(c, q, nq, d_prev, d_next, d_status, d_err, false, d_counts, count_stride);
}

int psn_lk_track_device(psn_lk_ctx *c, const psn_lk_query *q, int nq, const float *d_prev, float *d_next,
                        uint8_t *d_status, float *d_err) {
    if (!c || (nq > 0 && (!q || !d_prev || !d_next || !d_status)) || nq < 0) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return track_device_impl(c, q, nq, d_prev, d_next, d_status, d_err, false);
}

static int ensure_pts(psn_lk_ctx *c, size_t n) {
    if (c->d_pts_cap >= n) return PSN_LK_OK;
    for (void *p : {(void *)c->d_prev, (void *)c->d_next, (void *)c->d_err, (void *)c->d_status})
        if (p) (void)hipFree(p);
    c->d_prev = c->d_next = c->d_err = nullptr;
    c->d_status = nullptr;
    c->d_pts_cap = 0;
    size_t cap = std::max<size_t>(n, 1024);
    HIPCHK(c, hipMalloc(&c->d_prev, cap * 2 * sizeof(float)));
    HIPCHK(c, hipMalloc(&c->d_next, cap * 2 * sizeof(float)));
    HIPCHK(c, hipMalloc(&c->d_err, cap * sizeof(float)));
    HIPCHK(c, hipMalloc(&c->d_status, cap));
    c->d_pts_cap = cap;
    return PSN_LK_OK;
}

static int track_host_impl(psn_lk_ctx *c, const psn_lk_query *q, int nq, const float *prev_xy, float *next_xy,
                           uint8_t *status, float *err, bool allow_scratch) {
    size_t npts = 0;
    bool init_flow = false;
    for (int i = 0; i < nq; i++) {
        if (q[i].num_pts < 0 || q[i].first_pt < 0) return PSN_LK_ERR_ARG;
        npts = std::max(npts, (size_t)q[i].first_pt + q[i].num_pts);
        init_flow |= (q[i].params.flags & PSN_LK_USE_INITIAL_FLOW) != 0;
    }
    if (npts == 0) return track_device_impl(c, q, nq, nullptr, nullptr, nullptr, nullptr, allow_scratch);
    int rc = ensure_pts(c, npts);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_prev, prev_xy, npts * 2 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (init_flow) HIPCHK(c, hipMemcpyAsync(c->d_next, next_xy, npts * 2 * sizeof(float), hipMemcpyHostToDevice, c->stream));
    rc = track_device_impl(c, q, nq, c->d_prev, c->d_next, c->d_status, err ? c->d_err : nullptr, allow_scratch);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(next_xy, c->d_next, npts * 2 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(status, c->d_status, npts, hipMemcpyDeviceToHost, c->stream));
    if (err) HIPCHK(c, hipMemcpyAsync(err, c->d_err, npts * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PSN_LK_OK;
}

int psn_lk_track(psn_lk_ctx *c, const psn_lk_query *q, int nq, const float *prev_xy, float *next_xy, uint8_t *status,
                 float *err) {
    if (!c || nq < 0 || (nq > 0 && !q)) return PSN_LK_ERR_ARG;
    for (int i = 0; i < nq; i++)
        if (q[i].num_pts > 0 && (!prev_xy || !next_xy || !status)) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return track_host_impl(c, q, nq, prev_xy, next_xy, status, err, false);
}

int psn_calc_optical_flow_pyr_lk(psn_lk_ctx *c, const uint8_t *prev_img, const uint8_t *next_img, int stride,
                                 const float *prev_pts, float *next_pts, uint8_t *status, float *err, int npts,
                                 const psn_lk_params *params) {
    if (!c || !prev_img || !next_img || npts < 0 || stride < c->width) return PSN_LK_ERR_ARG;
    psn_lk_params p;
    if (params)
        p = *params;
    else
        psn_lk_default_params(&p);
    if (p.win_w <= 2 || p.win_h <= 2) return set_err(c, PSN_LK_ERR_WINSIZE, "winSize %dx%d <= 2", p.win_w, p.win_h);
    if (npts == 0) return PSN_LK_OK;  // calcOpticalFlowPyrLK releases outputs and returns
    if (!prev_pts || !next_pts || !status) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const int sa = c->user_slots, sb = c->user_slots + 1;
    int rc = push_host_impl(c, sa, prev_img, stride, 1);
    if (rc) return rc;
    rc = push_host_impl(c, sb, next_img, stride, 1);
    if (rc) return rc;
    psn_lk_query q;
    q.prev_slot = sa;
    q.next_slot = sb;
    q.first_pt = 0;
    q.num_pts = npts;
    q.params = p;
    return track_host_impl(c, &q, 1, prev_pts, next_pts, status, err, true);
}

int psn_lk_debug_set_variant(psn_lk_ctx *c, int key, int value) {
    if (!c) return PSN_LK_ERR_ARG;
    switch (key) {
    case PSN_LK_VARIANT_THREADS:
        if (value != 0 && value != 64 && value != 128 && value != 256 && value != 512) return PSN_LK_ERR_ARG;
        c->force_threads = value;
        return PSN_LK_OK;
    case PSN_LK_VARIANT_GENERIC: c->force_generic = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_ONEWAVE: c->onewave = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_BOX: c->box = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_TILED_LDS: c->tiled_lds = std::max(16 * 1024, std::min(value, 160 * 1024 - 1024)); return PSN_LK_OK;
    case PSN_LK_VARIANT_FUSED_HELPERS: c->fused_helpers = std::max(0, value); return PSN_LK_OK;
    case PSN_LK_VARIANT_LARGE: c->force_large = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_LG_LDS: c->lg_lds = std::max(4 * 1024, std::min(value, 160 * 1024 - 1024)); return PSN_LK_OK;
    case PSN_LK_VARIANT_LG_JR: c->lg_jr = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_ST_OVL: c->st_ovl = value != 0; return PSN_LK_OK;
    case PSN_LK_VARIANT_POISON_LDS: c->poison_lds = value != 0; return PSN_LK_OK;
    default: return PSN_LK_ERR_ARG;
    }
}

int psn_lk_debug_count_samples(psn_lk_ctx *c, int on) {
    if (!c) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    if (on) {
        if (!c->d_samples) HIPCHK(c, hipMalloc(&c->d_samples, sizeof(unsigned long long)));
        HIPCHK(c, hipDeviceSynchronize());
        HIPCHK(c, hipMemset(c->d_samples, 0, sizeof(unsigned long long)));
    }
    c->count_samples = on != 0;
    return PSN_LK_OK;
}

int psn_lk_debug_read_samples(psn_lk_ctx *c, unsigned long long *out) {
    if (!c || !out) return PSN_LK_ERR_ARG;
    *out = 0;
    if (!c->d_samples) return PSN_LK_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());  // launches of every stream the context was driven on
    HIPCHK(c, hipMemcpy(out, c->d_samples, sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return PSN_LK_OK;
}

int psn_lk_debug_set_stamps(psn_lk_ctx *c, void *d_stamps) {
    if (!c) return PSN_LK_ERR_ARG;
#ifdef PSN_LK_STAMPS
    c->d_stamps = (unsigned long long *)d_stamps;
    return PSN_LK_OK;
#else
    (void)d_stamps;
    return PSN_LK_ERR_UNSUPPORTED;
#endif
}

int psn_lk_read_level(psn_lk_ctx *c, int slot, int level, uint8_t *host, int stride) {
    if (!c || !host || slot < 0 || slot >= c->nslots || level < 0 || level >= c->nlevels) return PSN_LK_ERR_ARG;
    const LevelDev &L = c->h_slots[(size_t)slot * psn::kMaxLevels + level];
    if (stride < L.w) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = flush_pending(c);
    if (rc) return rc;
    rc = wait_slot_ready(c, slot);
    if (rc) return rc;
    HIPCHK(c, hipMemcpy2DAsync(host, stride, L.p, L.pitch, L.w, L.h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PSN_LK_OK;
}

// ---- GridFAST (include/psn_lk.h; kernels in psn_gridfast.hip) ----

void psn_gridfast_default_params(psn_gridfast_params *p) {
    if (!p) return;
    p->threshold = 10;  // FastFeatureDetector(10, true)
    p->nonmax = 1;
    p->max_total = 1000;  // GridAdaptedFeatureDetector(detector, 1000, 4, 4)
    p->grid_rows = 4;
    p->grid_cols = 4;
    p->cap = 100;  // PSN_2D_FEATURE_MAX_NUM_TRACK (PSNWhere_Tracker2D.cpp:13)
}

// nset sets of rois, set i = nrois[i] rois on ring slot slots[i], all sets'
// rois consecutive in `rois` and in the outputs; a launch covers up to
// kGfMaxRois rois of any sets (the shuffle key restarts at 0 per set).
static int gridfast_impl(psn_lk_ctx *c, int nset, const int *slots, const int *nrois, const int *rois,
                         const psn_gridfast_params *pp, uint32_t seed, float *d_xy, int *d_cnt, int *d_tot) {
    psn_gridfast_params p;
    if (pp)
        p = *pp;
    else
        psn_gridfast_default_params(&p);
    const int ncell = p.grid_rows * p.grid_cols;
    if (p.grid_rows <= 0 || p.grid_cols <= 0 || ncell > 256 || p.max_total > psn::kGfMaxTotal || p.cap < 0)
        return set_err(c, PSN_LK_ERR_ARG, "gridfast: grid %dx%d, max_total %d, cap %d", p.grid_rows, p.grid_cols,
                       p.max_total, p.cap);
    if ((c->width + p.grid_cols - 1) / p.grid_cols - 6 > psn::kGfMaxRegionW)
        return set_err(c, PSN_LK_ERR_UNSUPPORTED, "gridfast: cell width above %d", psn::kGfMaxRegionW + 6);
    int nroi = 0;
    std::vector<int> used;  // distinct slots with rois
    for (int i = 0; i < nset; i++) {
        const int slot = slots[i];
        if (slot < 0 || slot >= c->nslots || !c->filled[slot])
            return set_err(c, PSN_LK_ERR_SLOT, "slot %d not filled", slot);
        if (nrois[i] < 0) return set_err(c, PSN_LK_ERR_ARG, "gridfast: set %d has %d rois", i, nrois[i]);
        nroi += nrois[i];
        if (nrois[i] > 0 && std::find(used.begin(), used.end(), slot) == used.end()) used.push_back(slot);
    }
    if (nroi == 0) return PSN_LK_OK;
    for (int slot : used) {
        // the frame must be in the slot: a deferred build of it runs first
        if (c->pend && c->pend_slot == slot) {
            int rc = flush_pending(c);
            if (rc) return rc;
        }
        int rc = wait_slot_ready(c, slot);
        if (rc) return rc;
    }
    std::vector<const uint8_t *> roi_img((size_t)nroi);
    std::vector<int> roi_key((size_t)nroi);
    for (int i = 0, k = 0; i < nset; i++)
        for (int j = 0; j < nrois[i]; j++, k++) {
            roi_img[k] = c->h_slots[(size_t)slots[i] * psn::kMaxLevels].p;
            roi_key[k] = j;
        }
    psn::GridFastArgs a{};
    const LevelDev &L = c->h_slots[(size_t)used[0] * psn::kMaxLevels];
    a.w = L.w;
    a.h = L.h;
    a.pitch = L.pitch;
    a.threshold = std::min(std::max(p.threshold, 0), 255);
    a.nonmax = p.nonmax ? 1 : 0;
    a.grid_rows = p.grid_rows;
    a.grid_cols = p.grid_cols;
    // GridAdaptedFeatureDetector: nothing when maxTotalKeypoints < cells
    a.per_cell = p.max_total >= ncell ? p.max_total / ncell : 0;
    a.cap = p.cap;
    a.seed = seed;
    const size_t kp_need = (size_t)psn::kGfMaxRois * ncell * std::max(a.per_cell, 1);
    if (c->gf_kp_cap < kp_need) {
        if (c->d_gf_kp) (void)hipFree(c->d_gf_kp);
        c->d_gf_kp = nullptr;
        c->gf_kp_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_gf_kp, kp_need * sizeof(uint32_t)));
        c->gf_kp_cap = kp_need;
    }
    const size_t cnt_need = (size_t)psn::kGfMaxRois * ncell;
    if (c->gf_cnt_cap < cnt_need) {
        if (c->d_gf_cnt) (void)hipFree(c->d_gf_cnt);
        c->d_gf_cnt = nullptr;
        c->gf_cnt_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_gf_cnt, cnt_need * sizeof(int)));
        c->gf_cnt_cap = cnt_need;
    }
    a.cell_kp = c->d_gf_kp;
    a.cell_cnt = c->d_gf_cnt;
    for (int base = 0; base < nroi; base += psn::kGfMaxRois) {
        const int n = std::min(psn::kGfMaxRois, nroi - base);
        a.nroi = n;
        a.out_xy = d_xy + (size_t)base * p.cap * 2;
        a.out_count = d_cnt + base;
        a.out_total = d_tot ? d_tot + base : nullptr;
        // LDS plan: the widest region a (roi, cell) workgroup can see, the strip
        // height, the single-pass keypoint list (coordinates packed in 12 bits)
        int rw_max = 1;
        const int cell_w = (c->width + p.grid_cols - 1) / p.grid_cols - 6;
        for (int i = 0; i < n; i++) rw_max = std::max(rw_max, std::min(rois[4 * (size_t)(base + i) + 2], cell_w));
        a.rw_max = rw_max;
        a.list_cap = (c->width <= 4096 && c->height <= 4096) ? 4096 : 0;
        a.strip = 32;
        while (a.strip > 8 && psn::gridfast_lds_bytes(rw_max, a.strip, a.list_cap) > psn::kGfMaxLds) a.strip >>= 1;
        while (a.list_cap > 0 && psn::gridfast_lds_bytes(rw_max, a.strip, a.list_cap) > psn::kGfMaxLds) a.list_cap >>= 1;
        for (int i = 0; i < n; i++) {
            const int *r = rois + 4 * (size_t)(base + i);
            // clip to the image (cropWithSize already did for the reference's rois)
            int x0 = std::max(r[0], 0), y0 = std::max(r[1], 0);
            int x1 = std::min((long long)r[0] + r[2], (long long)c->width) > x0 ? (int)std::min((long long)r[0] + r[2], (long long)c->width) : x0;
            int y1 = std::min((long long)r[1] + r[3], (long long)c->height) > y0 ? (int)std::min((long long)r[1] + r[3], (long long)c->height) : y0;
            if (r[2] <= 0 || r[3] <= 0) x1 = x0, y1 = y0;
            a.rois[i] = make_int4(x0, y0, x1 - x0, y1 - y0);
            a.roi_img[i] = roi_img[base + i];
            a.roi_key[i] = roi_key[base + i];
        }
        HIPCHK(c, psn::launch_gridfast(a, c->stream));
    }
    // a later build into these slots waits for these reads
    return record_slots_free(c, used.data(), (int)used.size());
}

int psn_gridfast_detect_device(psn_lk_ctx *c, int slot, const int *rois, int nroi, const psn_gridfast_params *p,
                               uint32_t seed, float *d_out_xy, int *d_out_count, int *d_out_total) {
    if (!c || nroi < 0 || (nroi > 0 && (!rois || !d_out_xy || !d_out_count))) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return gridfast_impl(c, 1, &slot, &nroi, rois, p, seed, d_out_xy, d_out_count, d_out_total);
}

int psn_gridfast_detect_device_sets(psn_lk_ctx *c, int nset, const int *slots, const int *nrois, const int *rois,
                                    const psn_gridfast_params *p, uint32_t seed, float *d_out_xy, int *d_out_count,
                                    int *d_out_total) {
    if (!c || nset < 0 || (nset > 0 && (!slots || !nrois))) return PSN_LK_ERR_ARG;
    long long total = 0;
    for (int i = 0; i < nset; i++) total += std::max(nrois[i], 0);
    if (total > INT32_MAX || (total > 0 && (!rois || !d_out_xy || !d_out_count))) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return gridfast_impl(c, nset, slots, nrois, rois, p, seed, d_out_xy, d_out_count, d_out_total);
}

int psn_gridfast_detect(psn_lk_ctx *c, int slot, const int *rois, int nroi, const psn_gridfast_params *pp,
                        uint32_t seed, float *out_xy, int *out_count, int *out_total) {
    if (!c || nroi < 0 || (nroi > 0 && (!rois || !out_xy || !out_count))) return PSN_LK_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    psn_gridfast_params p;
    if (pp)
        p = *pp;
    else
        psn_gridfast_default_params(&p);
    if (nroi == 0 || p.cap < 0) return gridfast_impl(c, 1, &slot, &nroi, rois, &p, seed, nullptr, nullptr, nullptr);
    const size_t xy_need = (size_t)nroi * std::max(p.cap, 1) * 2;
    if (c->gf_out_cap < xy_need) {
        if (c->d_gf_xy) (void)hipFree(c->d_gf_xy);
        c->d_gf_xy = nullptr;
        c->gf_out_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_gf_xy, xy_need * sizeof(float)));
        c->gf_out_cap = xy_need;
    }
    if (c->gf_nroi_cap < nroi) {
        for (int **q : {&c->d_gf_oc, &c->d_gf_ot})
            if (*q) (void)hipFree(*q), *q = nullptr;
        c->gf_nroi_cap = 0;
        HIPCHK(c, hipMalloc(&c->d_gf_oc, (size_t)nroi * sizeof(int)));
        HIPCHK(c, hipMalloc(&c->d_gf_ot, (size_t)nroi * sizeof(int)));
        c->gf_nroi_cap = nroi;
    }
    int rc = gridfast_impl(c, 1, &slot, &nroi, rois, &p, seed, c->d_gf_xy, c->d_gf_oc, c->d_gf_ot);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(out_count, c->d_gf_oc, (size_t)nroi * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (out_total)
        HIPCHK(c, hipMemcpyAsync(out_total, c->d_gf_ot, (size_t)nroi * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (p.cap > 0)
        HIPCHK(c, hipMemcpyAsync(out_xy, c->d_gf_xy, (size_t)nroi * p.cap * 2 * sizeof(float), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PSN_LK_OK;
}

}  // extern "C"

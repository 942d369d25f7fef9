// capi.hip — the extern "C" boundary of libfir_hip.so (declared in include/fir_hip.h).
//
// Host-pointer entries own a per-device cache of device buffers and one non-blocking
// stream per device (grown on demand, never shrunk; guarded by a per-device mutex, so
// calls are reentrant across devices and serialised per device).  They are synchronous:
// H2D copy, kernel, D2H copy, stream synchronise.  Device-pointer entries (_dev) only
// enqueue on the caller's stream and never allocate or synchronise, so they can be
// captured in a hipGraph.  No C++ exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fir1d_reg_launch.h"
#include "fir_hip.h"
#include "fir_launch.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return fail(FIR_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct DeviceBuf {
    void* ptr = nullptr;
    size_t cap = 0;
};

struct DeviceState {
    std::mutex mu;
    bool init = false;
    hipStream_t stream = nullptr;
    hipStream_t stream_d2h = nullptr;  // the chunked host path's device-to-host copies
    static constexpr int kChunks = 8;
    hipEvent_t chunk_ev[kChunks] = {};  // the chunked host path's per-chunk kernel events
    DeviceBuf in, out;
    void* pin_in = nullptr;   // small calls: pinned host staging the kernel reads / writes directly
    void* pin_out = nullptr;
    size_t pin_cap = 0;
    std::vector<hipEvent_t> plane_ev;  // the image-batch entries: one per output plane (grow-only)
    hipEvent_t tev[4] = {};            // ... and their timing events (H2D start / end, kernels end, D2H end)
};

std::mutex g_devs_mu;
std::vector<std::unique_ptr<DeviceState>> g_devs;

int ensure(DeviceBuf& b, size_t bytes) {
    if (bytes <= b.cap) return FIR_OK;
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.cap = 0;
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    hipError_t e = hipMalloc(&b.ptr, want);
    if (e != hipSuccess) {
        b.ptr = nullptr;
        return fail(FIR_ENOMEM, std::string("hipMalloc(") + std::to_string(want) + "): " + hipGetErrorString(e));
    }
    b.cap = want;
    return FIR_OK;
}

// Puts the calling thread's current device back on scope exit: a host entry that runs on
// `device` must not move the caller's (e.g. PyTorch's) current device.
struct DeviceRestore {
    int prev = -1;
    DeviceRestore() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceRestore() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Validates `device`, makes it current, and returns its state (locked by the caller).
int device_state(int device, DeviceState** out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(FIR_ENODEV, std::string("no HIP device available: ") + (e != hipSuccess ? hipGetErrorString(e) : "0 devices"));
    if (device < 0 || device >= n)
        return fail(FIR_ENODEV, "device " + std::to_string(device) + " out of range (" + std::to_string(n) + " devices)");
    {
        std::lock_guard<std::mutex> lk(g_devs_mu);
        if ((int)g_devs.size() < n) {
            g_devs.reserve(n);
            while ((int)g_devs.size() < n) g_devs.emplace_back(new DeviceState());
        }
    }
    HIP_TRY(hipSetDevice(device));
    *out = g_devs[device].get();
    return FIR_OK;
}

int init_locked(DeviceState* st, int device) {
    if (st->init) return FIR_OK;
    hipDeviceProp_t p;
    HIP_TRY(hipGetDeviceProperties(&p, device));
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
        return fail(FIR_ENODEV, std::string("device ") + std::to_string(device) + " is " + p.gcnArchName +
                                    "; libfir_hip is built for gfx950 (MI355X) only");
    if (!st->stream) HIP_TRY(hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking));
    if (!st->stream_d2h) HIP_TRY(hipStreamCreateWithFlags(&st->stream_d2h, hipStreamNonBlocking));
    for (hipEvent_t& ev : st->chunk_ev)
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (hipEvent_t& ev : st->tev)
        if (!ev) HIP_TRY(hipEventCreate(&ev));
    st->init = true;
    return FIR_OK;
}

size_t in_size(int in_dtype) { return in_dtype == FIR_IN_I16 ? 2 : 1; }
size_t out_size(int stage) { return stage == FIR_OUT_I32 ? 4 : 1; }

// Small calls (the reference's callers run the model once per image row: 4.5 KB) skip both DMA
// copies: the input is memcpy'd into pinned host memory, the kernel reads it and writes its
// output there over PCIe (zero-copy), one stream synchronise, one memcpy out.  Measured per
// 4499-sample row (tools/row_call_latency.py): 40.5 us with the two pageable DMA copies.
// FIR_SMALL_CALLS=0 turns it off.
constexpr size_t kSmallCallBytes = size_t(1) << 20;  // in + out

bool small_calls_on() {
    static const bool on = [] {
        const char* e = std::getenv("FIR_SMALL_CALLS");
        return !(e && e[0] == '0');
    }();
    return on;
}

int ensure_pinned(DeviceState* st, size_t bytes) {
    if (bytes <= st->pin_cap) return FIR_OK;
    if (st->pin_in) (void)hipHostFree(st->pin_in);
    if (st->pin_out) (void)hipHostFree(st->pin_out);
    st->pin_in = st->pin_out = nullptr;
    st->pin_cap = 0;
    const size_t want = std::max(bytes, size_t(64) << 10);
    hipError_t e = hipHostMalloc(&st->pin_in, want, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(&st->pin_out, want, hipHostMallocDefault);
    if (e != hipSuccess) {
        if (st->pin_in) (void)hipHostFree(st->pin_in);
        st->pin_in = nullptr;
        return fail(FIR_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    st->pin_cap = want;
    return FIR_OK;
}

// Run `launch(dx, dy, stream)` between an H2D copy of `in_bytes` and a D2H copy of `out_bytes`
// (taken from byte `out_skip` of the device output).  The device buffers hold at least
// in_cap / out_cap bytes (scratch after the input, outputs not copied back).
template <typename F>
int run_host(int device, const void* x, size_t in_bytes, void* y, size_t out_bytes, F launch, size_t out_skip = 0,
             size_t in_cap = 0, size_t out_cap = 0, bool small_ok = false) {
    DeviceRestore restore;
    DeviceState* st = nullptr;
    int rc = device_state(device, &st);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(st->mu);
    rc = init_locked(st, device);
    if (rc) return rc;
    if (small_ok && out_skip == 0 && in_cap == 0 && out_cap == 0 && in_bytes + out_bytes <= kSmallCallBytes &&
        small_calls_on()) {
        if ((rc = ensure_pinned(st, std::max(in_bytes, out_bytes)))) return rc;
        std::memcpy(st->pin_in, x, in_bytes);
        std::string err;
        rc = launch(st->pin_in, st->pin_out, st->stream, &err);
        if (rc) {
            (void)hipStreamSynchronize(st->stream);
            return fail(rc, err);
        }
        HIP_TRY(hipStreamSynchronize(st->stream));
        std::memcpy(y, st->pin_out, out_bytes);
        return FIR_OK;
    }
    if ((rc = ensure(st->in, std::max(in_bytes, in_cap))) || (rc = ensure(st->out, std::max(out_skip + out_bytes, out_cap))))
        return rc;
    HIP_TRY(hipMemcpyAsync(st->in.ptr, x, in_bytes, hipMemcpyHostToDevice, st->stream));
    std::string err;
    rc = launch(st->in.ptr, st->out.ptr, st->stream, &err);
    if (rc) {
        (void)hipStreamSynchronize(st->stream);
        return fail(rc, err);
    }
    HIP_TRY(hipMemcpyAsync(y, (char*)st->out.ptr + out_skip, out_bytes, hipMemcpyDeviceToHost, st->stream));
    HIP_TRY(hipStreamSynchronize(st->stream));
    return FIR_OK;
}

// Large fir1d_fixed_rows host calls in kChunks pieces so the two PCIe directions overlap: this
// thread issues chunk i's H2D and then chunk i-1's kernel on `stream` (a single row's segment
// reads its right halo from chunk i, already staged); a second host thread issues chunk i-1's
// D2H on `stream_d2h` behind that kernel's event (a pageable D2H blocks its issuing thread).
// Chunk boundaries: row blocks for images (block starts kept 16-byte aligned so every chunk
// stays on the register kernel), and for one long row whole frames (`ch` samples) rounded to
// the register kernel's wave tile, so every interior segment is one halo-reading launch
// (halos inside the staged input, zero at the signal ends).  A u8 in-place call stays
// correct: chunk i's output is copied back only after chunk i+1's input left the host.
// FIR_HOST_CHUNKED=0 turns it off.
constexpr int kChunks = DeviceState::kChunks;
constexpr size_t kChunkedMinBytes = size_t(64) << 20;

bool use_chunked(int64_t rows, int64_t n, int in_dtype) {
    static const bool on = [] {
        const char* e = std::getenv("FIR_HOST_CHUNKED");
        return !(e && e[0] == '0');
    }();
    return on && (rows == 1 || rows >= kChunks) && (size_t)n * in_size(in_dtype) >= kChunkedMinBytes;
}

int64_t gcd64(int64_t a, int64_t b) {
    while (b) {
        const int64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// Chunk boundaries b[0..kChunks] in samples (see above); false when some chunk would be too
// short to hold its halos (the caller then runs the call unchunked).
bool chunk_bounds(int64_t rows, int64_t width, int ch, int in_dtype, int stage, int taps, int64_t b[kChunks + 1]) {
    const int64_t rowlen = width * ch, n = rows * rowlen;
    b[0] = 0;
    b[kChunks] = n;
    if (rows > 1) {
        const int64_t minsz = (int64_t)std::min(in_size(in_dtype), out_size(stage));
        const int64_t ra = 16 / gcd64(16, rowlen * minsz % 16);  // rows per 16-byte-aligned block start
        const int64_t units = rows / ra;
        if (units < kChunks) return false;
        for (int i = 1; i < kChunks; ++i) b[i] = units * i / kChunks * ra * rowlen;
        return true;
    }
    const int64_t tile = fir::reg_tile_samples(in_dtype == FIR_IN_U8);
    const int64_t g = tile / gcd64(tile, ch) * ch;  // lcm(tile, ch) samples
    const int64_t units = n / g;
    if (units < kChunks) return false;
    for (int i = 1; i < kChunks; ++i) b[i] = units * i / kChunks * g;
    const int64_t halo = (int64_t)(taps - 1) * ch;
    for (int i = 0; i < kChunks; ++i)
        if (b[i + 1] - b[i] < halo) return false;
    return true;
}

int run_host_chunked(int device, const void* x, int in_dtype, int64_t rows, int64_t width, int ch,
                     const int32_t* hq, int taps, int frac, int acc, int stage, void* y) {
    const size_t isz = in_size(in_dtype), osz = out_size(stage);
    const int64_t n = rows * width * ch;
    int64_t b[kChunks + 1];
    if (!chunk_bounds(rows, width, ch, in_dtype, stage, taps, b))
        return run_host(device, x, (size_t)n * isz, y, (size_t)n * osz, [&](void* dx, void* dy, hipStream_t s, std::string* err) {
            return fir::launch_fir1d_rows(dx, in_dtype, rows, width, ch, hq, taps, frac, acc, stage, dy, s, err);
        });
    DeviceRestore restore;
    DeviceState* st = nullptr;
    int rc = device_state(device, &st);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(st->mu);
    if ((rc = init_locked(st, device))) return rc;
    if ((rc = ensure(st->in, (size_t)n * isz)) || (rc = ensure(st->out, (size_t)n * osz))) return rc;
    const int64_t hl = (int64_t)(taps - 1 - taps / 2) * ch;
    char* dx = (char*)st->in.ptr;
    char* dy = (char*)st->out.ptr;
    hipEvent_t* ev = st->chunk_ev;
    std::mutex mu;
    std::condition_variable cv;
    int ready = 0;  // kernels whose event is recorded (kChunks + 1: abort)
    hipError_t d2h_err = hipSuccess;
    std::thread d2h([&] {
        (void)hipSetDevice(device);
        for (int i = 0; i < kChunks; ++i) {
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return ready > i; });
                if (ready > kChunks) return;
            }
            hipError_t e = hipStreamWaitEvent(st->stream_d2h, ev[i], 0);
            if (e == hipSuccess)
                e = hipMemcpyAsync((char*)y + b[i] * osz, dy + b[i] * osz, (size_t)(b[i + 1] - b[i]) * osz,
                                   hipMemcpyDeviceToHost, st->stream_d2h);
            if (e != hipSuccess) {
                d2h_err = e;
                return;
            }
        }
    });
    auto post = [&](int v) {
        {
            std::lock_guard<std::mutex> g(mu);
            ready = v;
        }
        cv.notify_one();
    };
    std::string err;
    hipError_t e = hipSuccess;
    auto kernel = [&](int i) -> int {
        int r;
        if (rows > 1)
            r = fir::launch_fir1d_rows(dx + b[i] * isz, in_dtype, (b[i + 1] - b[i]) / (width * ch), width, ch, hq, taps,
                                       frac, acc, stage, dy + b[i] * osz, st->stream, &err);
        else
            r = fir::launch_fir1d_segment(dx + b[i] * isz, in_dtype, (b[i + 1] - b[i]) / ch, ch, hq, taps, frac, acc,
                                          stage, i ? dx + (b[i] - hl) * isz : nullptr,
                                          i + 1 < kChunks ? dx + b[i + 1] * isz : nullptr, dy + b[i] * osz,
                                          st->stream, &err);
        if (r) return r;
        e = hipEventRecord(ev[i], st->stream);
        if (e != hipSuccess) return FIR_EHIP;
        post(i + 1);
        return FIR_OK;
    };
    for (int i = 0; i <= kChunks && !rc; ++i) {
        if (i < kChunks) {
            e = hipMemcpyAsync(dx + b[i] * isz, (const char*)x + b[i] * isz, (size_t)(b[i + 1] - b[i]) * isz,
                               hipMemcpyHostToDevice, st->stream);
            if (e != hipSuccess) rc = FIR_EHIP;
        }
        if (!rc && i > 0) rc = kernel(i - 1);
    }
    if (rc) post(kChunks + 1);
    d2h.join();
    // Every copy already queued must land before returning, on success or failure: the caller
    // may free `y`, and the next call reuses st->out.
    const hipError_t sync_d2h = hipStreamSynchronize(st->stream_d2h);
    (void)hipStreamSynchronize(st->stream);
    if (rc == FIR_EHIP && err.empty()) return fail(rc, std::string("chunked host path: ") + hipGetErrorString(e));
    if (rc) return fail(rc, err);
    if (d2h_err != hipSuccess) return fail(FIR_EHIP, std::string("chunked host path D2H: ") + hipGetErrorString(d2h_err));
    if (sync_d2h != hipSuccess) return fail(FIR_EHIP, std::string("chunked host path D2H: ") + hipGetErrorString(sync_d2h));
    return FIR_OK;
}

bool mul_ok(int64_t a, int64_t b, int64_t* out) {
    if (a < 0 || b < 0) return false;
    if (a != 0 && b > INT64_MAX / a) return false;
    *out = a * b;
    return true;
}

// The image-batch host entries (fir1d_fixed_images_multi, fir1d_ideal_images_multi): the stage's
// whole set of images goes to the device in one run of H2D copies (each image on a 256-byte
// boundary of the device input buffer), `launch(dx, dy, stream, err)` runs every kernel of the
// stage on those copies (output plane p on a 256-byte boundary of the device output buffer:
// planes start on whole cache lines), then each plane comes back by its own D2H copy, largest
// first, with an event behind it.  `ready(ctx, p)` is called on this thread as soon as plane p is
// in host memory, while the later planes are still in flight, so the caller can write plane p out
// (np.save) under the remaining copies; with pinned host buffers (fir_host_alloc) every copy is a
// DMA that needs no host thread.  timing_ms (optional): FIR_TIMING_SLOTS values, see fir_hip.h.
using PlaneReady = void (*)(void*, int);

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

template <typename F>
int run_host_images(int device, int n, const void* const* xs, const std::vector<size_t>& in_bytes, int np,
                    void* const* ys, const std::vector<size_t>& out_bytes, F launch, PlaneReady ready, void* ctx,
                    double* timing_ms) {
    const auto t_host0 = std::chrono::steady_clock::now();
    DeviceRestore restore;
    DeviceState* st = nullptr;
    int rc = device_state(device, &st);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(st->mu);
    if ((rc = init_locked(st, device))) return rc;
    std::vector<size_t> in_off(n), out_off(np);
    size_t in_total = 0, out_total = 0;
    for (int i = 0; i < n; ++i) {
        in_off[i] = in_total;
        in_total += align256(in_bytes[i]);
    }
    for (int p = 0; p < np; ++p) {
        out_off[p] = out_total;
        out_total += align256(out_bytes[p]);
    }
    if ((rc = ensure(st->in, std::max<size_t>(in_total, 256))) || (rc = ensure(st->out, std::max<size_t>(out_total, 256))))
        return rc;
    while ((int)st->plane_ev.size() < np) {
        hipEvent_t ev = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        st->plane_ev.push_back(ev);
    }
    std::vector<const void*> dx(n);
    std::vector<void*> dy(np);
    for (int i = 0; i < n; ++i) dx[i] = (const char*)st->in.ptr + in_off[i];
    for (int p = 0; p < np; ++p) dy[p] = (char*)st->out.ptr + out_off[p];
    hipStream_t s = st->stream;
    // every copy and kernel already queued must finish before an error return: the caller may
    // free its buffers, and the next call reuses the device buffers
    auto bail = [&](int code, const std::string& msg) {
        (void)hipStreamSynchronize(s);
        return fail(code, msg);
    };
    hipError_t e = hipSuccess;
    if (timing_ms) e = hipEventRecord(st->tev[0], s);
    for (int i = 0; i < n && e == hipSuccess; ++i)
        if (in_bytes[i]) e = hipMemcpyAsync((void*)dx[i], xs[i], in_bytes[i], hipMemcpyHostToDevice, s);
    if (e == hipSuccess && timing_ms) e = hipEventRecord(st->tev[1], s);
    if (e != hipSuccess) return bail(FIR_EHIP, std::string("image upload: ") + hipGetErrorString(e));
    std::string err;
    if ((rc = launch(dx.data(), dy.data(), s, &err))) return bail(rc, err);
    if (timing_ms && (e = hipEventRecord(st->tev[2], s)) != hipSuccess)
        return bail(FIR_EHIP, std::string("hipEventRecord: ") + hipGetErrorString(e));
    // largest planes first: their writes (the caller's longest) start earliest, under the copies
    // of the small ones
    std::vector<int> order(np);
    for (int p = 0; p < np; ++p) order[p] = p;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return out_bytes[a] > out_bytes[b]; });
    for (int k = 0; k < np && e == hipSuccess; ++k) {
        const int p = order[k];
        if (out_bytes[p]) e = hipMemcpyAsync(ys[p], dy[p], out_bytes[p], hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(st->plane_ev[k], s);
    }
    if (e == hipSuccess && timing_ms) e = hipEventRecord(st->tev[3], s);
    if (e != hipSuccess) return bail(FIR_EHIP, std::string("plane download: ") + hipGetErrorString(e));
    for (int k = 0; k < np && ready; ++k) {
        if ((e = hipEventSynchronize(st->plane_ev[k])) != hipSuccess)
            return bail(FIR_EHIP, std::string("plane download: ") + hipGetErrorString(e));
        ready(ctx, order[k]);
    }
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(FIR_EHIP, std::string("image batch: ") + hipGetErrorString(e));
    if (timing_ms) {
        float ms[3] = {0, 0, 0};
        for (int k = 0; k < 3; ++k)
            if ((e = hipEventElapsedTime(&ms[k], st->tev[k], st->tev[k + 1])) != hipSuccess)
                return fail(FIR_EHIP, std::string("hipEventElapsedTime: ") + hipGetErrorString(e));
        for (int k = 0; k < 3; ++k) timing_ms[k] = ms[k];
        timing_ms[3] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
    }
    return FIR_OK;
}

// Sizes of a batch of images (rows[i] x widths[i] x ch samples), FIR_EINVAL naming the image when
// one is impossible or a pointer it needs is NULL.
int image_sizes(int n, const void* const* xs, const int64_t* rows, const int64_t* widths, int64_t ch, int filters,
                void* const* ys, std::vector<int64_t>* samples) {
    if (n < 0) return fail(FIR_EINVAL, "images must be >= 0");
    if (filters < 1) return fail(FIR_EINVAL, "filters must be >= 1");
    if (n > 0 && (!xs || !rows || !widths || !ys)) return fail(FIR_EINVAL, "image arrays must not be NULL");
    samples->assign(n, 0);
    for (int i = 0; i < n; ++i) {
        int64_t rw = 0, s = 0;
        if (!mul_ok(rows[i], widths[i], &rw) || !mul_ok(rw, ch, &s))
            return fail(FIR_EINVAL, "image " + std::to_string(i) + ": invalid rows/width/channels");
        bool null = !xs[i];
        for (int f = 0; f < filters; ++f) null |= !ys[(size_t)i * filters + f];
        if (s && null) return fail(FIR_EINVAL, "image " + std::to_string(i) + ": x and its output planes must not be NULL");
        (*samples)[i] = s;
    }
    return FIR_OK;
}

}  // namespace

extern "C" {

int fir_abi_version(void) { return FIR_HIP_ABI_VERSION; }

#ifndef FIR_BUILD_ID
#define FIR_BUILD_ID "unknown"
#endif
const char* fir_build_id(void) { return FIR_BUILD_ID; }

const char* fir_last_error(void) { return g_err.c_str(); }

int fir_device_count(int* count) {
    if (!count) return fail(FIR_EINVAL, "count must not be NULL");
    *count = 0;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return fail(FIR_ENODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *count = n;
    return FIR_OK;
}

int fir1d_fixed_rows(const void* x, int in_dtype, int64_t rows, int64_t width, int channels, const int32_t* hq,
                     int taps, int frac_bits, int acc_bits, int out_stage, void* y, int device) {
    try {
        int64_t n = 0, rw = 0;
        if (channels < 1 || !mul_ok(rows, width, &rw) || !mul_ok(rw, channels, &n))
            return fail(FIR_EINVAL, "invalid rows/width/channels");
        if (n == 0) {
            std::string err;
            // still validate the scalar arguments
            int rc = fir::launch_fir1d_rows(nullptr, in_dtype, 0, 0, channels, hq, taps, frac_bits, acc_bits,
                                            out_stage, nullptr, nullptr, &err);
            return rc ? fail(rc, err) : FIR_OK;
        }
        if (!x || !y) return fail(FIR_EINVAL, "x and y must not be NULL");
        if (use_chunked(rows, n, in_dtype)) {
            // scalar arguments validated by a zero-size launch first, as the unchunked path does
            std::string err;
            int rc = fir::launch_fir1d_rows(nullptr, in_dtype, 0, 0, channels, hq, taps, frac_bits, acc_bits,
                                            out_stage, nullptr, nullptr, &err);
            if (rc) return fail(rc, err);
            return run_host_chunked(device, x, in_dtype, rows, width, channels, hq, taps, frac_bits, acc_bits,
                                    out_stage, y);
        }
        return run_host(device, x, (size_t)n * in_size(in_dtype), y, (size_t)n * out_size(out_stage),
                        [&](void* dx, void* dy, hipStream_t s, std::string* err) {
                            return fir::launch_fir1d_rows(dx, in_dtype, rows, width, channels, hq, taps, frac_bits,
                                                          acc_bits, out_stage, dy, s, err);
                        }, 0, 0, 0, true);
    } catch (const std::exception& ex) {
        return fail(FIR_EHIP, std::string("internal error: ") + ex.what());
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_rows_sharded(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                             const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage, void* y,
                             const int* devices, int ndev) {
    try {
        if (ndev < 1 || !devices) return fail(FIR_EINVAL, "devices must list ndev >= 1 device ids");
        int64_t n = 0, rw = 0;
        if (channels < 1 || !mul_ok(rows, width, &rw) || !mul_ok(rw, channels, &n))
            return fail(FIR_EINVAL, "invalid rows/width/channels");
        {
            std::string err;  // the scalar arguments, once
            int rc = fir::launch_fir1d_rows(nullptr, in_dtype, 0, 0, channels, hq, taps, frac_bits, acc_bits,
                                            out_stage, nullptr, nullptr, &err);
            if (rc) return fail(rc, err);
        }
        if (n == 0) return FIR_OK;
        if (!x || !y) return fail(FIR_EINVAL, "x and y must not be NULL");
        const size_t isz = in_size(in_dtype), osz = out_size(out_stage);
        struct Shard {
            int64_t in0, rows, width;  // launch: rows x width (x channels) samples from sample in0
            int64_t skip, out0, len;   // copy outputs [skip, skip + len) of the launch to y[out0 ...]
        };
        std::map<int, std::vector<Shard>> by_dev;
        if (rows > 1) {  // independent rows: contiguous row blocks
            for (int i = 0; i < ndev; ++i) {
                const int64_t r0 = rows * i / ndev, r1 = rows * (i + 1) / ndev;
                if (r1 > r0)
                    by_dev[devices[i]].push_back({r0 * width * channels, r1 - r0, width, 0, r0 * width * channels,
                                                  (r1 - r0) * width * channels});
            }
        } else {  // one row: segments widened by their halos (zero padding only at the row ends)
            const int64_t hl = taps - 1 - taps / 2, hr = taps / 2;
            for (int i = 0; i < ndev; ++i) {
                const int64_t s0 = width * i / ndev, s1 = width * (i + 1) / ndev;
                if (s1 <= s0) continue;
                const int64_t a = std::max<int64_t>(0, s0 - hl), b = std::min<int64_t>(width, s1 + hr);
                by_dev[devices[i]].push_back({a * channels, 1, b - a, (s0 - a) * channels, s0 * channels,
                                              (s1 - s0) * channels});
            }
        }
        std::vector<std::thread> workers;
        std::vector<int> rcs(by_dev.size(), FIR_OK);
        std::vector<std::string> msgs(by_dev.size());
        size_t wi = 0;
        for (auto& kv : by_dev) {
            const int dev = kv.first;
            const std::vector<Shard>* list = &kv.second;
            int* rc = &rcs[wi];
            std::string* msg = &msgs[wi];
            ++wi;
            workers.emplace_back([=]() noexcept {
                try {
                    for (const Shard& sh : *list) {
                        const int64_t cnt = sh.rows * sh.width * channels;
                        *rc = run_host(
                            dev, (const char*)x + sh.in0 * isz, (size_t)cnt * isz, (char*)y + sh.out0 * osz,
                            (size_t)sh.len * osz,
                            [&](void* dx, void* dy, hipStream_t s, std::string* err) {
                                return fir::launch_fir1d_rows(dx, in_dtype, sh.rows, sh.width, channels, hq, taps,
                                                              frac_bits, acc_bits, out_stage, dy, s, err);
                            },
                            (size_t)sh.skip * osz, 0, (size_t)cnt * osz);
                        if (*rc) {
                            *msg = g_err;  // thread-local: this worker's message
                            return;
                        }
                    }
                } catch (const std::exception& ex) {  // never let an exception end the process
                    *rc = FIR_EHIP;
                    *msg = std::string("internal error: ") + ex.what();
                } catch (...) {
                    *rc = FIR_EHIP;
                    *msg = "internal error";
                }
            });
        }
        for (auto& t : workers) t.join();
        for (size_t i = 0; i < rcs.size(); ++i)
            if (rcs[i]) return fail(rcs[i], msgs[i]);
        return FIR_OK;
    } catch (const std::exception& ex) {
        return fail(FIR_EHIP, std::string("internal error: ") + ex.what());
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_rows_dev(const void* x_dev, int in_dtype, int64_t rows, int64_t width, int channels,
                         const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage, void* y_dev,
                         void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir1d_rows(x_dev, in_dtype, rows, width, channels, hq, taps, frac_bits, acc_bits,
                                        out_stage, y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_rows_multi(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                           const int32_t* hq, int taps, int filters, int frac_bits, int acc_bits, int out_stage,
                           void* y, int device) {
    try {
        int64_t n = 0, rw = 0, nf = 0;
        if (channels < 1 || filters < 1 || !mul_ok(rows, width, &rw) || !mul_ok(rw, channels, &n) ||
            !mul_ok(n, filters, &nf))
            return fail(FIR_EINVAL, "invalid rows/width/channels/filters");
        if (n == 0) {
            std::string err;
            int rc = fir::launch_fir1d_rows_multi(nullptr, in_dtype, 0, 0, channels, hq, taps, filters, frac_bits,
                                                  acc_bits, out_stage, nullptr, nullptr, &err);
            return rc ? fail(rc, err) : FIR_OK;
        }
        if (!x || !y) return fail(FIR_EINVAL, "x and y must not be NULL");
        return run_host(device, x, (size_t)n * in_size(in_dtype), y, (size_t)nf * out_size(out_stage),
                        [&](void* dx, void* dy, hipStream_t s, std::string* err) {
                            return fir::launch_fir1d_rows_multi(dx, in_dtype, rows, width, channels, hq, taps, filters,
                                                                frac_bits, acc_bits, out_stage, dy, s, err);
                        }, 0, 0, 0, true);
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_rows_multi_dev(const void* x_dev, int in_dtype, int64_t rows, int64_t width, int channels,
                               const int32_t* hq, int taps, int filters, int frac_bits, int acc_bits, int out_stage,
                               void* y_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir1d_rows_multi(x_dev, in_dtype, rows, width, channels, hq, taps, filters, frac_bits,
                                              acc_bits, out_stage, y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_images_multi_dev(int n_images, const void* const* x_devs, const int64_t* rows, const int64_t* widths,
                                 int in_dtype, int channels, const int32_t* hq, int taps, int filters, int frac_bits,
                                 int acc_bits, int out_stage, void* const* y_planes, void* stream) {
    try {
        std::string err;
        int64_t rw = 0, n = 0;
        for (int i = 0; i < n_images && rows && widths; ++i)
            if (!mul_ok(rows[i], widths[i], &rw) || !mul_ok(rw, channels < 1 ? 1 : channels, &n))
                return fail(FIR_EINVAL, "image " + std::to_string(i) + ": invalid rows/width/channels");
        int rc = fir::launch_fir1d_images_multi(n_images, x_devs, rows, widths, in_dtype, channels, hq, taps, filters,
                                                frac_bits, acc_bits, out_stage, y_planes, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_images_multi(int n_images, const void* const* xs, const int64_t* rows, const int64_t* widths,
                             int in_dtype, int channels, const int32_t* hq, int taps, int filters, int frac_bits,
                             int acc_bits, int out_stage, void* const* y_planes, int device, fir_plane_ready_fn ready,
                             void* ready_ctx, double* timing_ms) {
    try {
        if (channels < 1) return fail(FIR_EINVAL, "channels must be >= 1");
        std::vector<int64_t> samples;
        int rc = image_sizes(n_images, xs, rows, widths, channels, filters, y_planes, &samples);
        if (rc) return rc;
        {
            std::string err;  // the scalar arguments, before any device work
            rc = fir::launch_fir1d_rows_multi(nullptr, in_dtype, 0, 0, channels, hq, taps, filters, frac_bits, acc_bits,
                                              out_stage, nullptr, nullptr, &err);
            if (rc) return fail(rc, err);
        }
        int64_t total = 0;
        for (int64_t s : samples) total += s;
        if (total == 0) return FIR_OK;
        const size_t isz = in_size(in_dtype), osz = out_size(out_stage);
        std::vector<size_t> ib(n_images), ob((size_t)n_images * filters);
        for (int i = 0; i < n_images; ++i) {
            ib[i] = (size_t)samples[i] * isz;
            for (int f = 0; f < filters; ++f) ob[(size_t)i * filters + f] = (size_t)samples[i] * osz;
        }
        return run_host_images(
            device, n_images, xs, ib, n_images * filters, y_planes, ob,
            [&](const void* const* dx, void* const* dy, hipStream_t s, std::string* err) {
                return fir::launch_fir1d_images_multi(n_images, dx, rows, widths, in_dtype, channels, hq, taps, filters,
                                                      frac_bits, acc_bits, out_stage, dy, s, err);
            },
            ready, ready_ctx, timing_ms);
    } catch (const std::exception& ex) {
        return fail(FIR_EHIP, std::string("internal error: ") + ex.what());
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_edges_dev(const void* x_dev, int in_dtype, int64_t n, int channels, const int32_t* hq, int taps,
                          int frac_bits, int acc_bits, int out_stage, const void* halo_left_dev,
                          const void* halo_right_dev, void* y_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir1d_edges(x_dev, in_dtype, n, channels, hq, taps, frac_bits, acc_bits, out_stage,
                                         halo_left_dev, halo_right_dev, y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_fixed_segment_dev(const void* x_dev, int in_dtype, int64_t n, int channels, const int32_t* hq, int taps,
                            int frac_bits, int acc_bits, int out_stage, const void* halo_left_dev,
                            const void* halo_right_dev, void* y_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir1d_segment(x_dev, in_dtype, n, channels, hq, taps, frac_bits, acc_bits, out_stage,
                                           halo_left_dev, halo_right_dev, y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir2d_fixed_frames(const uint8_t* x, int64_t frames, int64_t height, int64_t width, const int32_t* hq,
                       int tap_rows, int tap_cols, int frac_bits, int acc_bits, int out_stage, void* y, int device) {
    try {
        int64_t n = 0, hw = 0;
        if (!mul_ok(height, width, &hw) || !mul_ok(hw, frames, &n)) return fail(FIR_EINVAL, "invalid frames/height/width");
        if (n == 0) {
            std::string err;
            int rc = fir::launch_fir2d(nullptr, 0, 0, 0, hq, tap_rows, tap_cols, frac_bits, acc_bits, out_stage,
                                       nullptr, nullptr, &err);
            return rc ? fail(rc, err) : FIR_OK;
        }
        if (!x || !y) return fail(FIR_EINVAL, "x and y must not be NULL");
        return run_host(device, x, (size_t)n, y, (size_t)n * out_size(out_stage),
                        [&](void* dx, void* dy, hipStream_t s, std::string* err) {
                            return fir::launch_fir2d((const uint8_t*)dx, frames, height, width, hq, tap_rows, tap_cols,
                                                     frac_bits, acc_bits, out_stage, dy, s, err);
                        });
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir2d_fixed(const uint8_t* x, int64_t height, int64_t width, const int32_t* hq, int tap_rows, int tap_cols,
                int frac_bits, int acc_bits, int out_stage, void* y, int device) {
    return fir2d_fixed_frames(x, 1, height, width, hq, tap_rows, tap_cols, frac_bits, acc_bits, out_stage, y, device);
}

int fir2d_fixed_frames_dev(const uint8_t* x_dev, int64_t frames, int64_t height, int64_t width, const int32_t* hq,
                           int tap_rows, int tap_cols, int frac_bits, int acc_bits, int out_stage, void* y_dev,
                           void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir2d(x_dev, frames, height, width, hq, tap_rows, tap_cols, frac_bits, acc_bits, out_stage,
                                   y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir2d_fixed_dev(const uint8_t* x_dev, int64_t height, int64_t width, const int32_t* hq, int tap_rows,
                    int tap_cols, int frac_bits, int acc_bits, int out_stage, void* y_dev, void* stream) {
    return fir2d_fixed_frames_dev(x_dev, 1, height, width, hq, tap_rows, tap_cols, frac_bits, acc_bits, out_stage, y_dev,
                                  stream);
}

int fir1d_ideal_rows(const uint8_t* x, int64_t rows, int64_t width, const double* h, int taps, double* y,
                     int device) {
    try {
        int64_t n = 0;
        if (!mul_ok(rows, width, &n)) return fail(FIR_EINVAL, "invalid rows/width");
        if (n == 0) {
            std::string err;
            int rc = fir::launch_fir1d_ideal(nullptr, 0, 0, h, taps, nullptr, nullptr, &err);
            return rc ? fail(rc, err) : FIR_OK;
        }
        if (!x || !y) return fail(FIR_EINVAL, "x and y must not be NULL");
        return run_host(device, x, (size_t)n, y, (size_t)n * 8, [&](void* dx, void* dy, hipStream_t s, std::string* err) {
            return fir::launch_fir1d_ideal((const uint8_t*)dx, rows, width, h, taps, (double*)dy, s, err);
        }, 0, 0, 0, true);
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_ideal_rows_dev(const uint8_t* x_dev, int64_t rows, int64_t width, const double* h, int taps,
                         double* y_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_fir1d_ideal(x_dev, rows, width, h, taps, y_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir1d_ideal_images_multi(int n_images, const uint8_t* const* xs, const int64_t* rows, const int64_t* widths,
                             const double* h, int taps, int filters, double* const* y_planes, int device,
                             fir_plane_ready_fn ready, void* ready_ctx, double* timing_ms) {
    try {
        std::vector<int64_t> samples;
        int rc = image_sizes(n_images, (const void* const*)xs, rows, widths, 1, filters, (void* const*)y_planes,
                             &samples);
        if (rc) return rc;
        for (int f = 0; f < filters; ++f) {  // every filter's taps, before any device work
            std::string err;
            rc = fir::launch_fir1d_ideal(nullptr, 0, 0, h ? h + (size_t)f * (taps > 0 ? taps : 0) : nullptr, taps,
                                         nullptr, nullptr, &err);
            if (rc) return fail(rc, "filter " + std::to_string(f) + ": " + err);
        }
        int64_t total = 0;
        for (int64_t s : samples) total += s;
        if (total == 0) return FIR_OK;
        std::vector<size_t> ib(n_images), ob((size_t)n_images * filters);
        for (int i = 0; i < n_images; ++i) {
            ib[i] = (size_t)samples[i];
            for (int f = 0; f < filters; ++f) ob[(size_t)i * filters + f] = (size_t)samples[i] * sizeof(double);
        }
        return run_host_images(
            device, n_images, (const void* const*)xs, ib, n_images * filters, (void* const*)y_planes, ob,
            [&](const void* const* dx, void* const* dy, hipStream_t s, std::string* err) {
                for (int i = 0; i < n_images; ++i) {
                    if (!samples[i]) continue;
                    for (int f = 0; f < filters; ++f) {
                        const int r = fir::launch_fir1d_ideal((const uint8_t*)dx[i], rows[i], widths[i],
                                                              h + (size_t)f * taps, taps,
                                                              (double*)dy[(size_t)i * filters + f], s, err);
                        if (r) return r;
                    }
                }
                return (int)FIR_OK;
            },
            ready, ready_ctx, timing_ms);
    } catch (const std::exception& ex) {
        return fail(FIR_EHIP, std::string("internal error: ") + ex.what());
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_host_alloc(int64_t bytes, void** out) {
    try {
        if (!out || bytes < 0) return fail(FIR_EINVAL, "invalid arguments");
        *out = nullptr;
        if (bytes == 0) return FIR_OK;
        hipError_t e = hipHostMalloc(out, (size_t)bytes, hipHostMallocPortable);
        if (e != hipSuccess) {
            *out = nullptr;
            return fail(FIR_ENOMEM, "hipHostMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
        }
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_host_free(void* p) {
    if (!p) return FIR_OK;
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? FIR_OK : fail(FIR_EHIP, std::string("hipHostFree: ") + hipGetErrorString(e));
}

int64_t fir_metrics_work_bytes(int64_t n) { return (int64_t)fir::metrics_work_bytes(n); }

int fir_compare_metrics(const double* ideal, const void* fixed, int fixed_dtype, int64_t n, double* out,
                        int device) {
    try {
        if (n < 0 || !out || (n > 0 && (!ideal || !fixed))) return fail(FIR_EINVAL, "invalid arguments");
        const int es = fir::metrics_dtype_size(fixed_dtype);
        if (!es) return fail(FIR_EINVAL, "unknown fixed dtype");
        DeviceRestore restore;
        DeviceState* st = nullptr;
        int rc = device_state(device, &st);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(st->mu);
        if ((rc = init_locked(st, device))) return rc;
        const size_t ib = (size_t)n * 8, fb = (size_t)n * es;
        const size_t fo = (ib + 255) / 256 * 256;
        if ((rc = ensure(st->in, fo + fb + 1)) || (rc = ensure(st->out, fir::metrics_work_bytes(n) + 256))) return rc;
        char* din = (char*)st->in.ptr;
        if (n > 0) {
            HIP_TRY(hipMemcpyAsync(din, ideal, ib, hipMemcpyHostToDevice, st->stream));
            HIP_TRY(hipMemcpyAsync(din + fo, fixed, fb, hipMemcpyHostToDevice, st->stream));
        }
        double* dout = (double*)st->out.ptr;
        std::string err;
        rc = fir::launch_metrics((const double*)din, din + fo, fixed_dtype, n, dout, (char*)st->out.ptr + 256,
                                 st->stream, &err);
        if (rc) {
            (void)hipStreamSynchronize(st->stream);
            return fail(rc, err);
        }
        HIP_TRY(hipMemcpyAsync(out, dout, 9 * sizeof(double), hipMemcpyDeviceToHost, st->stream));
        HIP_TRY(hipStreamSynchronize(st->stream));
        if (out[8] != 0.0) return fail(FIR_EHIP, "metrics: the in-kernel hand-off timed out");
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_compare_metrics_dev(const double* ideal_dev, const void* fixed_dev, int fixed_dtype, int64_t n,
                            double* out_dev, void* work_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_metrics(ideal_dev, fixed_dev, fixed_dtype, n, out_dev, work_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int64_t fir_restore_work_bytes(void) { return (int64_t)fir::restore_work_bytes(); }

int fir_restore_u8(const double* a, int64_t n, int policy, uint8_t* out, int device) {
    try {
        if (n < 0 || (n > 0 && (!a || !out))) return fail(FIR_EINVAL, "invalid arguments");
        if (n == 0) {
            std::string err;
            int rc = fir::launch_restore_u8(nullptr, 0, policy, nullptr, nullptr, nullptr, &err);
            return rc ? fail(rc, err) : FIR_OK;
        }
        const size_t ab = (size_t)n * 8, wo = (ab + 255) / 256 * 256;
        // device input = a, then the normalize scratch
        return run_host(device, a, ab, out, (size_t)n, [&](void* da, void* dout, hipStream_t s, std::string* err) {
            return fir::launch_restore_u8((const double*)da, n, policy, (uint8_t*)dout, (char*)da + wo, s, err);
        }, 0, wo + fir::restore_work_bytes());
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_restore_u8_dev(const double* a_dev, int64_t n, int policy, uint8_t* out_dev, void* work_dev, void* stream) {
    try {
        std::string err;
        int rc = fir::launch_restore_u8(a_dev, n, policy, out_dev, work_dev, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

// ---- xGMI peer halos (fir_hip.h) --------------------------------------------------------
static_assert(sizeof(hipIpcMemHandle_t) == FIR_IPC_HANDLE_BYTES, "IPC handle size");

namespace {
std::mutex g_ipc_mu;
std::map<void*, void*> g_ipc_base;  // pointer handed out by fir_ipc_import -> mapped base
}  // namespace

int fir_ipc_export(const void* dev_ptr, void* handle_out, int64_t* offset_out) {
    try {
        if (!dev_ptr || !handle_out || !offset_out) return fail(FIR_EINVAL, "NULL argument");
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dev_ptr);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipMemGetAddressRange: ") + hipGetErrorString(e));
        hipIpcMemHandle_t h;
        e = hipIpcGetMemHandle(&h, (void*)base);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
        std::memcpy(handle_out, &h, sizeof(h));
        *offset_out = (int64_t)((const char*)dev_ptr - (const char*)base);
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_ipc_import(const void* handle, int64_t offset, int device, void** dev_ptr_out) {
    try {
        if (!handle || !dev_ptr_out || offset < 0) return fail(FIR_EINVAL, "invalid argument");
        *dev_ptr_out = nullptr;
        DeviceRestore restore;
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return fail(FIR_ENODEV, std::string("hipSetDevice: ") + hipGetErrorString(e));
        hipIpcMemHandle_t h;
        std::memcpy(&h, handle, sizeof(h));
        void* base = nullptr;
        e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
        void* p = (char*)base + offset;
        std::lock_guard<std::mutex> g(g_ipc_mu);
        g_ipc_base[p] = base;
        *dev_ptr_out = p;
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_ipc_close(void* dev_ptr) {
    try {
        void* base = nullptr;
        {
            std::lock_guard<std::mutex> g(g_ipc_mu);
            auto it = g_ipc_base.find(dev_ptr);
            if (it == g_ipc_base.end()) return fail(FIR_EINVAL, "pointer was not returned by fir_ipc_import");
            base = it->second;
            g_ipc_base.erase(it);
        }
        hipError_t e = hipIpcCloseMemHandle(base);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipIpcCloseMemHandle: ") + hipGetErrorString(e));
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_device_bus_id(int device, char* out, int len) {
    try {
        if (!out || len < 16) return fail(FIR_EINVAL, "out must hold at least 16 bytes");
        out[0] = 0;
        hipError_t e = hipDeviceGetPCIBusId(out, len, device);
        if (e != hipSuccess) return fail(FIR_ENODEV, std::string("hipDeviceGetPCIBusId: ") + hipGetErrorString(e));
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_peer_access(int device, const char* peer_bus_id, int* can) {
    try {
        if (!peer_bus_id || !can) return fail(FIR_EINVAL, "NULL argument");
        *can = 0;
        int peer = -1;
        if (hipDeviceGetByPCIBusId(&peer, peer_bus_id) != hipSuccess || peer < 0) {
            (void)hipGetLastError();  // not visible to this process: no kernel path to it
            return FIR_OK;
        }
        if (peer == device) {
            *can = 1;
            return FIR_OK;
        }
        int ok = 0;
        hipError_t e = hipDeviceCanAccessPeer(&ok, device, peer);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipDeviceCanAccessPeer: ") + hipGetErrorString(e));
        *can = ok ? 1 : 0;
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_peer_atomics(int device, const char* peer_bus_id, int* can) {
    try {
        if (!peer_bus_id || !can) return fail(FIR_EINVAL, "NULL argument");
        *can = 0;
        int peer = -1;
        if (hipDeviceGetByPCIBusId(&peer, peer_bus_id) != hipSuccess || peer < 0) {
            (void)hipGetLastError();
            return FIR_OK;
        }
        if (peer == device) {
            *can = 1;
            return FIR_OK;
        }
        int ok = 0;
        hipError_t e = hipDeviceGetP2PAttribute(&ok, hipDevP2PAttrNativeAtomicSupported, device, peer);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipDeviceGetP2PAttribute: ") + hipGetErrorString(e));
        *can = ok ? 1 : 0;
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int64_t fir_halo_mailbox_bytes(int64_t halo_left_bytes, int64_t halo_right_bytes) {
    if (halo_left_bytes < 0 || halo_right_bytes < 0) return -1;
    return fir::halo_mailbox_bytes(halo_left_bytes, halo_right_bytes);
}

int fir_halo_mailbox_init_dev(void* mailbox_dev, int64_t bytes, int64_t halo_left_bytes, int64_t halo_right_bytes,
                              void* stream) {
    try {
        std::string err;
        int rc = fir::launch_halo_mailbox_init(mailbox_dev, bytes, halo_left_bytes, halo_right_bytes,
                                               (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_halo_gate_dev(const void* x_dev, int64_t seg_bytes, int64_t halo_left_bytes, int64_t halo_right_bytes,
                      void* mailbox_dev, const void* left_mailbox_dev, const void* right_mailbox_dev,
                      void* halo_left_dev, void* halo_right_dev, int32_t* status_dev, double timeout_s,
                      void* stream) {
    try {
        std::string err;
        int rc = fir::launch_halo_gate(x_dev, seg_bytes, halo_left_bytes, halo_right_bytes, mailbox_dev,
                                       left_mailbox_dev, right_mailbox_dev, halo_left_dev, halo_right_dev, status_dev,
                                       timeout_s, (hipStream_t)stream, &err);
        return rc ? fail(rc, err) : FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

int fir_peek(const void* dev_ptr, void* host_out, int64_t bytes) {
    try {
        if (bytes < 0 || (bytes > 0 && (!dev_ptr || !host_out))) return fail(FIR_EINVAL, "invalid argument");
        if (bytes == 0) return FIR_OK;
        hipError_t e = hipMemcpy(host_out, dev_ptr, (size_t)bytes, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return fail(FIR_EHIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
        return FIR_OK;
    } catch (...) {
        return fail(FIR_EHIP, "internal error");
    }
}

}  // extern "C"

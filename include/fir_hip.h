/*
 * fir_hip.h — C ABI of libfir_hip.so, the MI355X (gfx950) fixed-point FIR path.
 *
 * Plain C types only (pointers, sizes, ints); no exceptions cross this boundary.
 * Every entry returns a fir_status; on failure fir_last_error() (thread-local)
 * holds the message.  Argument validation that the reference performs in Python
 * (ValueError texts of fir_1d_ref.py:9-33 / fir_1d_fixed_ref.py:39-72) stays in the
 * Python host layer; these entries only reject structurally impossible calls
 * (FIR_EINVAL) and report HIP/device failures (FIR_EHIP / FIR_ENODEV).
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   fir1d_fixed_rows      the per-row loop of fir_1d/sim/vector/gen_fixed_output.py:34-60
 *                         (_run_fixed_rowwise), each row being a call of
 *                         fir_1d/model/python/fir_1d_fixed_ref.py:12-130 (fir_1d_fixed_golden)
 *                         after its host-side prep (:33-81); one call per image instead of
 *                         one per row.  A single row is the fir_1d_fixed_golden call itself.
 *   fir1d_fixed_rows_dev  same, device buffers, asynchronous on a caller stream (bench,
 *                         sharded driver, graph capture).
 *   fir1d_fixed_rows_multi[_dev] the same for F coefficient sets over one input: the loop
 *                         over a bank's filters in gen_fixed_output.py:92-105, one read of x
 *                         for up to 4 filters.
 *   fir1d_fixed_images_multi_dev the stage's loop over images x coefficient sets
 *                         (gen_fixed_output.py:88-107): up to 8 images x 4 filters per launch,
 *                         each output plane its own device buffer (ABI 5).
 *   fir1d_fixed_images_multi  the same stage from host memory, as generate_fixed_{3,5}tap_output_vector
 *                         (gen_fixed_output.py:88-107) runs it: every pending image uploaded once,
 *                         one batch launch, each output plane downloaded on its own and handed to
 *                         the caller (np.save) while the rest are in flight (ABI 6).
 *   fir1d_ideal_images_multi  the ideal stage's loop (gen_ideal_output.py:75-86) the same way:
 *                         one upload per image for all of its coefficient sets (ABI 6).
 *   fir1d_fixed_edges_dev recomputes the first (L-1-L/2) and last (L/2) outputs of a
 *                         segment from neighbour halo samples (multi-GPU sharding, SURVEY
 *                         §8(e)); no reference counterpart (the reference is one process).
 *   fir2d_fixed[_dev]     fir_2d/model/cpp/CMakeLists.txt is empty in the reference; the
 *                         2-D semantics are the build's.
 *   fir1d_ideal_rows[_dev] fir_1d/model/python/fir_1d_ref.py:43-65 (fir_1d_ideal) per row as
 *                         in fir_1d/sim/vector/gen_ideal_output.py:37-50.
 *   fir_compare_metrics   fir_1d/sim/vector/gen_3tap_compare_report.py:67-112 (_compute_metrics).
 *   fir1d_fixed_rows_sharded  the `fir1d_sharded(..., ndev)` entry of SURVEY §8(b): one call
 *                         spread over several devices of this process (rows split, or a long
 *                         row split into segments with their halos); the reference has no
 *                         multi-device form.
 *   fir_restore_u8[_dev]  fir_1d/sim/vector/restore_images.py:51-64 (_to_u8_clip,
 *                         _to_u8_normalized), the array half of the restore stage.
 *
 * Arithmetic (all fixed entries): y[n] = stage(round(wrap_acc(sum_k hq[k] * x[n - k + L/2])))
 *   wrap_acc: two's-complement wrap to acc_bits (fir_1d_fixed_ref.py:110-115)
 *   round:    (acc + 2^(frac_bits-1)) >> frac_bits, arithmetic (:118-120)
 *   stage:    FIR_OUT_U8_SAT clamps to [0,255] (:123-126); FIR_OUT_I32 keeps the int32 value.
 * Samples outside a row are zero (:99-104) unless halo buffers are supplied.
 */
#ifndef FIR_HIP_H
#define FIR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FIR_HIP_ABI_VERSION 6
/* Tap counts: any length up to FIR_MAX_TAPS (1-D taps; 2-D tap_rows * tap_cols), like the
 * reference's Python loop (fir_1d_fixed_ref.py:83-107, fir_1d_ref.py:49-63); the bound is the
 * int taps argument and device memory (4 B per tap), not the arithmetic.  Sums are exact as the
 * reference's unbounded Python ints: mod 2^64 for acc_bits < 64, 64-bit while sum|hq| * max|x|
 * < 2^63, 128-bit otherwise (ABI 4; < 2^127 for every legal input). */
#define FIR_MAX_TAPS (1 << 30)

typedef enum {
    FIR_OK = 0,
    FIR_EINVAL = 1, /* structurally invalid arguments (null pointer, bad enum, size) */
    FIR_EHIP = 2,   /* a HIP runtime call failed */
    FIR_ENODEV = 3, /* no usable gfx950 device / device index out of range */
    FIR_ENOMEM = 4  /* device allocation failed */
} fir_status;

typedef enum { FIR_IN_U8 = 0, FIR_IN_I16 = 1 } fir_in_dtype;
typedef enum { FIR_OUT_U8_SAT = 0, FIR_OUT_I32 = 1 } fir_out_stage;

/* Library / device queries.  fir_build_id: a hash of the sources the library was built from
 * (csrc/, csrc/Makefile and this header); the Python loader refuses a library whose id differs
 * from the sources beside it (a stale build). */
int fir_abi_version(void);
const char* fir_build_id(void);
const char* fir_last_error(void);
int fir_device_count(int* count);

/* ---- 1-D fixed-point FIR over independent rows (a1, a4, a6, a7) -------------------
 * x: rows x (width*channels) samples of in_dtype, C-contiguous; channels > 1 means
 * interleaved channels (complex int16 = 2) filtered independently with the same real
 * taps.  hq: `taps` quantized coefficients (host memory, int32).  y: same shape, uint8
 * (FIR_OUT_U8_SAT) or int32 (FIR_OUT_I32).  1 <= frac_bits, 1 <= acc_bits.
 * Host-pointer form: synchronous (H2D, kernel, D2H) on `device`. */
int fir1d_fixed_rows(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                     const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage,
                     void* y, int device);

/* Device-pointer form: enqueued on `stream` (hipStream_t; NULL = default stream of the
 * current device); returns after the launch, not after completion. */
int fir1d_fixed_rows_dev(const void* x_dev, int in_dtype, int64_t rows, int64_t width,
                         int channels, const int32_t* hq, int taps, int frac_bits, int acc_bits,
                         int out_stage, void* y_dev, void* stream);

/* F filters of `taps` taps each over the same x: hq is F x taps (row-major), y holds F
 * consecutive output planes shaped like x (plane f at y + f * rows*width*channels elements).
 * Results are identical to F calls of fir1d_fixed_rows; u8 input reads x once per 4 filters. */
int fir1d_fixed_rows_multi(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                           const int32_t* hq, int taps, int filters, int frac_bits, int acc_bits, int out_stage,
                           void* y, int device);
int fir1d_fixed_rows_multi_dev(const void* x_dev, int in_dtype, int64_t rows, int64_t width, int channels,
                               const int32_t* hq, int taps, int filters, int frac_bits, int acc_bits,
                               int out_stage, void* y_dev, void* stream);

/* The pipeline's stage over a set of images (replaces the per-image loop of
 * fir_1d/sim/vector/gen_fixed_output.py:88-107, which runs _run_fixed_rowwise once per image and
 * coefficient set and keeps each output as its own array): image i is rows[i] x widths[i] x
 * channels samples at x_devs[i]; its output for filter f (shaped like the image) at
 * y_planes[i * filters + f], each plane its own buffer.  Results are identical to one
 * fir1d_fixed_rows_dev call per (image, filter); every image is checked before anything launches
 * (an error names the image).  u8 -> sat-u8 banks of one channel go out as ONE launch per 8
 * images and 4 filters (device pointers, stream-ordered, returns after the launches).  Planes
 * that start on 128 bytes are written in whole cache lines (16 bytes off: 18.7 vs 16.2 us for the
 * golden images' stage, 238 vs 181 us for a 2^28-sample bank; profiles/r05/pipeline_batch_ab.txt). */
int fir1d_fixed_images_multi_dev(int n_images, const void* const* x_devs, const int64_t* rows,
                                 const int64_t* widths, int in_dtype, int channels, const int32_t* hq,
                                 int taps, int filters, int frac_bits, int acc_bits, int out_stage,
                                 void* const* y_planes, void* stream);

/* ---- host-memory image batches (ABI 6) ---------------------------------------------
 * The stage drivers' entries: the pipeline stages read every image from a .npy file and write
 * every output plane to its own .npy file, so the device work of a stage is one upload of its
 * images, its kernels, and one download per plane.  fir1d_fixed_images_multi runs
 * fir1d_fixed_images_multi_dev's launches (same layout of xs / rows / widths / y_planes, host
 * pointers) on `device`: the images are copied to the device back to back (256-byte aligned), the
 * planes come back one D2H copy each, largest first (ties in y_planes order), and
 * `ready(ready_ctx, p)` (optional) is called once per plane p, on the calling thread, as soon as it
 * is in host memory -- while the later planes are still being copied -- so the caller can write it
 * out under the remaining copies (the largest writes start first).  `ready` must
 * not call this library for the same device.  Synchronous: every plane is in host memory when
 * the entry returns.  With host buffers from fir_host_alloc (page-locked) every copy is a DMA at
 * the PCIe rate; pageable buffers also work (staged by the runtime).  timing_ms (optional, NULL
 * to skip) receives FIR_TIMING_SLOTS values in milliseconds: [0] the uploads, [1] the kernels,
 * [2] the downloads (HIP events on the entry's stream), [3] the whole call on the host clock.
 * fir1d_ideal_images_multi: the float64 ideal model the same way; h holds `filters` sets of
 * `taps` coefficients (row-major), plane i * filters + f = image i under set f.
 * fir_host_alloc / fir_host_free: page-locked host memory usable by every device's copies
 * (hipHostMalloc, portable); bytes == 0 gives NULL. */
typedef void (*fir_plane_ready_fn)(void* ctx, int plane);
#define FIR_TIMING_SLOTS 4
int fir1d_fixed_images_multi(int n_images, const void* const* xs, const int64_t* rows, const int64_t* widths,
                             int in_dtype, int channels, const int32_t* hq, int taps, int filters, int frac_bits,
                             int acc_bits, int out_stage, void* const* y_planes, int device,
                             fir_plane_ready_fn ready, void* ready_ctx, double* timing_ms);
int fir1d_ideal_images_multi(int n_images, const uint8_t* const* xs, const int64_t* rows, const int64_t* widths,
                             const double* h, int taps, int filters, double* const* y_planes, int device,
                             fir_plane_ready_fn ready, void* ready_ctx, double* timing_ms);
int fir_host_alloc(int64_t bytes, void** out);
int fir_host_free(void* p);

/* Recompute the first (taps-1-taps/2)*channels and last (taps/2)*channels outputs of a
 * single-row segment of n*channels samples, reading out-of-segment samples from
 * halo_left_dev ((taps-1-taps/2)*channels samples preceding the segment) and
 * halo_right_dev ((taps/2)*channels samples following it); a NULL halo means zeros.
 * Used after fir1d_fixed_rows_dev when the segment is a shard of a longer signal. */
int fir1d_fixed_edges_dev(const void* x_dev, int in_dtype, int64_t n, int channels,
                          const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage,
                          const void* halo_left_dev, const void* halo_right_dev, void* y_dev,
                          void* stream);

/* One shard of a longer single-row signal, halos given: the same outputs as
 * fir1d_fixed_rows_dev followed by fir1d_fixed_edges_dev, in ONE register-kernel launch (the
 * halos stand in for the zero padding) when n*channels is a whole number of 16-byte vectors
 * and the buffers are 16-byte aligned; otherwise exactly those two launches.  The halos may
 * live in another GPU's HBM mapped by fir_ipc_import (read over xGMI). */
int fir1d_fixed_segment_dev(const void* x_dev, int in_dtype, int64_t n, int channels,
                            const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage,
                            const void* halo_left_dev, const void* halo_right_dev, void* y_dev,
                            void* stream);

/* One-process multi-device form of fir1d_fixed_rows.  `devices`
 * lists ndev device ids (repeats allowed: a device then runs its shards in turn).
 * rows > 1: contiguous blocks of rows, no exchange (rows are independent).
 * rows == 1: contiguous segments; each device receives its segment plus the
 * (taps-1-taps/2)*channels / (taps/2)*channels neighbour samples around it from the host
 * buffer, so no device-to-device exchange is needed.  One host thread per distinct
 * device; synchronous; results identical to fir1d_fixed_rows. */
int fir1d_fixed_rows_sharded(const void* x, int in_dtype, int64_t rows, int64_t width, int channels,
                             const int32_t* hq, int taps, int frac_bits, int acc_bits, int out_stage,
                             void* y, const int* devices, int ndev);

/* ---- 2-D fixed-point FIR (a8) ------------------------------------------------------
 * y[i,j] = stage(round(wrap(sum_m sum_n hq[m*tap_cols+n] * x[i-m+tap_rows/2][j-n+tap_cols/2])))
 * x: height x width uint8, zero padded at every frame edge. */
int fir2d_fixed(const uint8_t* x, int64_t height, int64_t width, const int32_t* hq, int tap_rows,
                int tap_cols, int frac_bits, int acc_bits, int out_stage, void* y, int device);
int fir2d_fixed_dev(const uint8_t* x_dev, int64_t height, int64_t width, const int32_t* hq,
                    int tap_rows, int tap_cols, int frac_bits, int acc_bits, int out_stage,
                    void* y_dev, void* stream);
/* A batch of `frames` (<= 65535) frames of height x width stored back to back, each filtered
 * on its own (zero padding at every frame edge), in ONE launch: identical to `frames` calls of
 * the single-frame entries.  A launch per 8192^2 frame leaves the chip idle at its start and end;
 * a batch of 4 such frames streams from HBM 12 % faster per frame (profiles/r02). */
int fir2d_fixed_frames(const uint8_t* x, int64_t frames, int64_t height, int64_t width, const int32_t* hq,
                       int tap_rows, int tap_cols, int frac_bits, int acc_bits, int out_stage, void* y,
                       int device);
int fir2d_fixed_frames_dev(const uint8_t* x_dev, int64_t frames, int64_t height, int64_t width,
                           const int32_t* hq, int tap_rows, int tap_cols, int frac_bits, int acc_bits,
                           int out_stage, void* y_dev, void* stream);

/* ---- float64 "ideal" model ----------------------------------------
 * y[r,n] = sum over k (in k order, products and sums rounded separately, zero terms for
 * padding) of h[k] * x[r, n - k + taps/2]; no output clamp.  x uint8 rows x width. */
int fir1d_ideal_rows(const uint8_t* x, int64_t rows, int64_t width, const double* h, int taps,
                     double* y, int device);
int fir1d_ideal_rows_dev(const uint8_t* x_dev, int64_t rows, int64_t width, const double* h,
                         int taps, double* y_dev, void* stream);

/* ---- fixed-vs-ideal comparison metrics -----------------------------
 * One pass over `n` samples of ideal (float64) and fixed outputs of `fixed_dtype` (the
 * reference takes any dtype: y_fixed.astype(np.float64), gen_3tap_compare_report.py:84-86;
 * its fixed stage writes uint8, FIR_DT_U8 is the bandwidth path).  out[9] =
 * {max|d|, sum|d|, sum d^2, sum d, #(fixed==0), #(fixed==255), #(ideal<0 or >255), n, status}
 * with d = float64(fixed) - ideal; the report ratios are these over n.  The float64 sums are
 * added in NumPy's order (8192-sample blocks summed pairwise, block sums in order), so they equal
 * the reference's np.mean values bit for bit; counts are exact; max|d| is NaN when any |d| is
 * (np.max propagates NaN).  `work_dev` of the _dev form holds at least fir_metrics_work_bytes(n)
 * bytes.  status (out[8]) is 0; 1 means the one-launch pass's in-kernel hand-off gave up waiting
 * (10 s after the launch starts, on the GPU's 100 MHz clock; no correct run comes near it): the
 * sums are then NaN, and fir_compare_metrics returns
 * FIR_EHIP.  ABI 4: the fixed dtype argument. */
typedef enum {
    FIR_DT_U8 = 0, FIR_DT_I8 = 1, FIR_DT_U16 = 2, FIR_DT_I16 = 3, FIR_DT_U32 = 4, FIR_DT_I32 = 5,
    FIR_DT_U64 = 6, FIR_DT_I64 = 7, FIR_DT_F16 = 8, FIR_DT_F32 = 9, FIR_DT_F64 = 10
} fir_num_dtype;
int64_t fir_metrics_work_bytes(int64_t n);
int fir_compare_metrics(const double* ideal, const void* fixed, int fixed_dtype, int64_t n, double* out,
                        int device);
int fir_compare_metrics_dev(const double* ideal_dev, const void* fixed_dev, int fixed_dtype, int64_t n,
                            double* out_dev, void* work_dev, void* stream);

/* ---- restore-stage u8 conversion -----------------------------------
 * out[i] = u8 of a[i] (float64), n samples:
 *   FIR_RESTORE_CLIP       clip(rint(a), 0, 255)                         (restore_images.py:51-54)
 *   FIR_RESTORE_NORMALIZE  0 if max <= min, else rint(clip((a - min) * (255 / (max - min)),
 *                          0, 255))                                        (:57-64)
 * rint rounds half to even; NaN maps to 0.  The _dev form needs fir_restore_work_bytes() of
 * device scratch (normalize only; may be NULL for clip); a and out 16-byte aligned. */
typedef enum { FIR_RESTORE_CLIP = 0, FIR_RESTORE_NORMALIZE = 1 } fir_restore_policy;
int64_t fir_restore_work_bytes(void);
int fir_restore_u8(const double* a, int64_t n, int policy, uint8_t* out, int device);
int fir_restore_u8_dev(const double* a_dev, int64_t n, int policy, uint8_t* out_dev, void* work_dev,
                       void* stream);

/* ---- xGMI peer halos for sharded segments ---------------------------
 * One process per GPU: each rank exports the device buffer holding its segment once, its
 * neighbours map it, and every step's edge kernel (fir1d_fixed_edges_dev) reads its
 * (taps-1)-sample halo straight out of the neighbours' HBM over xGMI -- no per-step message.
 * fir_ipc_export: an opaque FIR_IPC_HANDLE_BYTES-byte handle of the allocation containing
 *   dev_ptr, and dev_ptr's byte offset inside that allocation.
 * fir_ipc_import: map a handle exported by ANOTHER process on this node for kernels on
 *   `device`; *dev_ptr_out = mapped base + offset.  Release with fir_ipc_close(*dev_ptr_out).
 * fir_peek: synchronous copy of `bytes` device bytes (own or imported) to host memory.
 * fir_device_bus_id: the PCI bus id ("0000:05:00.0") of `device`, NUL-terminated in `out`.
 * fir_peer_access: *can = 1 when kernels on `device` may read the HBM of the GPU with PCI bus
 *   id `peer_bus_id` (the same GPU, or a peer visible to this process with peer access);
 *   0 when that GPU is not visible here or has no peer path.  Checked before any kernel
 *   reads a mapped neighbour (a mapping alone does not prove a kernel may read it).
 * fir_peer_atomics: *can = 1 when kernels on `device` may also perform atomics on that GPU's
 *   HBM (the same GPU, or hipDevP2PAttrNativeAtomicSupported); the halo gate below needs it. */
#define FIR_IPC_HANDLE_BYTES 64
int fir_device_bus_id(int device, char* out, int len);
int fir_peer_access(int device, const char* peer_bus_id, int* can);
int fir_peer_atomics(int device, const char* peer_bus_id, int* can);
int fir_ipc_export(const void* dev_ptr, void* handle_out, int64_t* offset_out);
int fir_ipc_import(const void* handle, int64_t offset, int device, void** dev_ptr_out);
int fir_ipc_close(void* dev_ptr);
int fir_peek(const void* dev_ptr, void* host_out, int64_t bytes);

/* ---- per-step ordering of the halo hand-off --------------------------
 * When every rank's segment changes from step to step, rank r must read the neighbours'
 * segments of THIS step.  Each rank owns a mailbox in its own HBM (zeroed once, exported with
 * fir_ipc_export, mapped by both neighbours with fir_ipc_import); every step, on the rank's
 * stream after the step's segment is written and before the FIR kernel that uses the halos,
 * fir_halo_gate_dev runs ONE wave that
 *   1. publishes the segment's first halo_right_bytes (its left neighbour's right halo) and
 *      last halo_left_bytes (its right neighbour's left halo) with this step's epoch,
 *   2. waits until both present neighbours have published the same epoch (at most timeout_s
 *      seconds; on expiry *status_dev = FIR_GATE_TIMEOUT, the halos are zeroed, and every later
 *      gate of this mailbox stops waiting and reports the same),
 *   3. copies the left neighbour's published tail into halo_left_dev (halo_left_bytes) and the
 *      right neighbour's published head into halo_right_dev (halo_right_bytes).
 * A NULL neighbour mailbox is a global end (no wait, halo untouched).  Mailbox words are only
 * touched by device atomics (performed at the memory side: coherent across XCDs and xGMI).
 * All ranks of a ring must use the same halo sizes and call the gate once per step.
 * fir_halo_mailbox_bytes: size of one mailbox; fir_halo_mailbox_init_dev: zero it on `stream`
 * and record the halo sizes its slots are laid out for (before it is exported; every rank's init
 * must complete before any neighbour's first gate).  A gate whose own or neighbours' mailboxes
 * were laid out for other halo sizes touches no slot: *status_dev = FIR_GATE_LAYOUT, halos zero.
 * Mailboxes must be 128-byte aligned; halo sizes below 2^31 bytes. */
#define FIR_GATE_TIMEOUT 1
#define FIR_GATE_LAYOUT 2
int64_t fir_halo_mailbox_bytes(int64_t halo_left_bytes, int64_t halo_right_bytes);
int fir_halo_mailbox_init_dev(void* mailbox_dev, int64_t bytes, int64_t halo_left_bytes, int64_t halo_right_bytes,
                              void* stream);
int fir_halo_gate_dev(const void* x_dev, int64_t seg_bytes, int64_t halo_left_bytes, int64_t halo_right_bytes,
                      void* mailbox_dev, const void* left_mailbox_dev, const void* right_mailbox_dev,
                      void* halo_left_dev, void* halo_right_dev, int32_t* status_dev, double timeout_s,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FIR_HIP_H */

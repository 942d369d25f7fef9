// fir_launch.h — internal launch functions (C++), wrapped by the C ABI in capi.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

namespace fir {

// Device copies of host tables (long tap sets, matrix-core tap fragments) on the current device
// (dev_tables.hip): cached by the exact bytes they are made from -- their content, or the inputs
// a derived table is built from, behind a kind tag (table_acquire builds the table with `fill`
// only on a miss) -- looked up by a 128-bit hash of those bytes and confirmed by comparing them
// (a hash collision is a miss, never another table), uploaded once (complete before the call
// returns).  Every acquire is a hold on the table for ONE launch, released by table_release after
// that launch is enqueued on `stream` (TableHold does it at scope exit): the cache frees a table
// only when no hold is outstanding and every launch that used it has completed; a table used
// inside a stream capture is kept for the process life.  nullptr + *err on failure.  The first use
// of a table cannot be captured in a hipGraph (warm up before capturing).
enum TableKind : uint8_t { kTableRaw = 1, kTableMfmaFrag = 2 };
struct TableHash {
    uint64_t a = 0xcbf29ce484222325ull, c = 0x84222325cbf29ce4ull;
    std::vector<uint8_t> src;  // every byte added: the identity the cache compares on a hash hit
    explicit TableHash(TableKind kind) { add_val(kind); }
    void add(const void* p, size_t n);
    template <typename T>
    void add_val(const T& v) { add(&v, sizeof(v)); }
};
const void* table_acquire(TableHash&& h, size_t bytes, const std::function<void(void*)>& fill, std::string* err);
void table_release(const void* d, hipStream_t stream, bool launched = true);
const void* device_table(const void* host, size_t bytes, std::string* err);  // table_acquire by content
struct TableHold {  // one launch's hold: released (its use recorded on `s`) when the scope ends
    const void* p;
    hipStream_t s;
    TableHold(const void* p_, hipStream_t s_) : p(p_), s(s_) {}
    TableHold(const TableHold&) = delete;
    TableHold& operator=(const TableHold&) = delete;
    ~TableHold() { table_release(p, s); }
};

// Enqueue the row-wise 1-D fixed FIR on `stream`; device pointers.  Returns fir_status.
int launch_fir1d_rows(const void* x, int in_dtype, int64_t rows, int64_t width, int ch, const int32_t* hq, int L,
                      int frac, int acc_bits, int stage, void* y, hipStream_t stream, std::string* err);

// Long filters (up to 64 taps, one channel, int16 taps, acc_bits <= 32): the LDS-window
// v_dot2 kernel (fir1d_lds.hip).  lds_path_ok says whether it applies.
// Long filters on the matrix cores (fir1d_mfma.hip): 2..64 int16 taps, one channel,
// acc_bits <= 32, one row or rows of a multiple of 8 samples, aligned buffers.
bool mfma_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total, int ch,
                  const int32_t* hq, int L, int frac, int acc_bits);
hipError_t launch_fir1d_mfma(const void* x, int in_dtype, int64_t rows, int64_t rowlen, int64_t total,
                             const int32_t* hq, int L, int frac, int acc_bits, int stage, void* y, hipStream_t s);
bool lds_path_ok(const void* x, const void* y, int in_dtype, int64_t rows, int64_t rowlen, int64_t total, int ch,
                 const int32_t* hq, int L, int frac, int acc_bits);
hipError_t launch_fir1d_lds(const void* x, int in_dtype, int64_t rows, int64_t rowlen, int64_t total,
                            const int32_t* hq, int L, int frac, int acc_bits, int stage, void* y, hipStream_t s);

// F filters of L taps (hq row-major F x L) over the same x; y = F consecutive output planes.
int launch_fir1d_rows_multi(const void* x, int in_dtype, int64_t rows, int64_t width, int ch, const int32_t* hq,
                            int L, int F, int frac, int acc_bits, int stage, void* y, hipStream_t stream,
                            std::string* err);
// n images, F filters each: output plane (i, f) at planes[i * F + f]; every image is checked
// before anything launches.  u8 -> sat-u8 banks of one channel on the register kernel go out as
// ONE launch per 8 images (and per 4 filters), the rest as launch_fir1d_rows per plane.
int launch_fir1d_images_multi(int n, const void* const* xs, const int64_t* rows, const int64_t* widths, int in_dtype,
                              int ch, const int32_t* hq, int L, int F, int frac, int acc_bits, int stage,
                              void* const* planes, hipStream_t stream, std::string* err);

// Recompute the halo-dependent edge outputs of a single-row segment.
int launch_fir1d_edges(const void* x, int in_dtype, int64_t n, int ch, const int32_t* hq, int L, int frac,
                       int acc_bits, int stage, const void* halo_left, const void* halo_right, void* y,
                       hipStream_t stream, std::string* err);

// A single-row shard with its halos: bulk + edges in one register-kernel launch when possible.
int launch_fir1d_segment(const void* x, int in_dtype, int64_t n, int ch, const int32_t* hq, int L, int frac,
                         int acc_bits, int stage, const void* halo_left, const void* halo_right, void* y,
                         hipStream_t stream, std::string* err);

// Per-step halo ordering for sharded segments (halo_gate.hip): mailbox size, its zeroing, and
// the one-wave gate kernel (publish own edges, wait for both neighbours' epoch, copy their
// edges into the local halo buffers).
int64_t halo_mailbox_bytes(int64_t hl_bytes, int64_t hr_bytes);
int launch_halo_mailbox_init(void* mailbox, int64_t bytes, int64_t hl_bytes, int64_t hr_bytes, hipStream_t stream,
                             std::string* err);
int launch_halo_gate(const void* x, int64_t seg_bytes, int64_t hl_bytes, int64_t hr_bytes, void* mailbox,
                     const void* left_mailbox, const void* right_mailbox, void* halo_left, void* halo_right,
                     int32_t* status, double timeout_s, hipStream_t stream, std::string* err);

// 2-D fixed FIR over `frames` uint8 frames of height x width stored back to back (one launch).
// 2-D u8 -> sat-u8 frames on the int8 matrix cores (fir2d_mfma.hip); hipErrorNotSupported when
// the shape, alignment or taps are outside its cover (the caller then takes fir2d_reg_kernel)
hipError_t launch_fir2d_mfma(const uint8_t* x, int64_t frames, int64_t H, int64_t W, const int32_t* hq, int R, int C,
                             int frac, int acc_bits, int stage, void* y, hipStream_t s);
int launch_fir2d(const uint8_t* x, int64_t frames, int64_t height, int64_t width, const int32_t* hq, int tap_rows,
                 int tap_cols, int frac, int acc_bits, int stage, void* y, hipStream_t stream, std::string* err);

// float64 ideal model over uint8 rows.
int launch_fir1d_ideal(const uint8_t* x, int64_t rows, int64_t width, const double* h, int L, double* y,
                       hipStream_t stream, std::string* err);

// Fixed-vs-ideal comparison metrics (one pass); `work` >= metrics_work_bytes(n).
size_t metrics_work_bytes(int64_t n);
int metrics_dtype_size(int fixed_dtype);  // bytes per element of a fir_num_dtype, 0 if unknown
int launch_metrics(const double* ideal, const void* fixed, int fixed_dtype, int64_t n, double* out, void* work,
                   hipStream_t stream, std::string* err);

// f64 -> u8 restore conversion (FIR_RESTORE_*); `work` >= restore_work_bytes() for normalize.
size_t restore_work_bytes();
int launch_restore_u8(const double* a, int64_t n, int policy, uint8_t* out, void* work, hipStream_t stream,
                      std::string* err);

}  // namespace fir

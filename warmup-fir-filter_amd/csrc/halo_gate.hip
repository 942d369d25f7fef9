// halo_gate.hip — per-step ordering of the halo hand-off between sharded ranks.
//
// A long signal is cut into one contiguous segment per rank (one process per GPU).  An L-tap
// filter makes rank r read the last HL samples of rank r-1 and the first HR samples of rank
// r+1 every step.  When the segments change from step to step (streaming), that read must see
// the neighbour's segment OF THIS STEP: not the previous one, and not the next one the
// neighbour may already be writing.  The gate orders it without any host round trip:
//
//   every rank owns a small mailbox in its own HBM, exported once over HIP IPC and mapped by
//   both neighbours.  Each step, ONE wave on each rank (this kernel, stream-ordered after
//   whatever produced the step's segment and before the FIR kernel):
//     1. copies its segment's first HR samples (the left neighbour's right halo) and last HL
//        samples (the right neighbour's left halo) into mailbox slot (e & 1), e = its step
//        count + 1, then writes e into that slot's epoch word;
//     2. waits until both neighbours' slot (e & 1) carries epoch e (bounded: on a timeout it
//        records FIR_GATE_TIMEOUT in its status word and stops waiting);
//     3. copies the neighbours' published samples into two local halo buffers, which the FIR
//        kernel (fir1d_fixed_segment_dev) then reads like any halo.
//   Two slots suffice: rank r rewrites slot (e & 1) at step e + 2 only after its own step e + 1
//   gate saw the neighbour's epoch e + 1, which the neighbour published after its step e gate
//   had finished reading slot (e & 1).  No cycle: a gate publishes before it waits, and step e's
//   publications depend only on every rank having finished step e - 1.
//
// Coherence: every mailbox word is written and read ONLY by device atomics at system scope
// (exchange / fetch_add of a runtime 0), which MI355X performs at the memory side, not in an L2 (the L2s are
// per XCD and not coherent with each other nor with a peer GPU's writes over xGMI).  A writer's
// returning atomics complete (s_waitcnt vmcnt(0)) before its epoch word is written; a reader
// issues its payload reads after its epoch read has returned the new value.  No plain load or
// store ever touches a mailbox line, so no cache can hold a stale copy of one.
//
// Mailbox layout (dwords; every field starts a 128-byte line):
//   [0]            the owner's gate count (steps published so far)
//   [1]            status: 0 ok, FIR_GATE_TIMEOUT after a wait gave up (later gates skip waiting)
//   [2], [3]       the halo sizes (HL, HR bytes) the slots are laid out for, written at init; a gate
//                  compares its own sizes with its mailbox's and both neighbours' before it
//                  computes any slot address (a mismatch would index past a smaller mailbox)
//   slot s at dword 32 + s * slot_dw:   [0] epoch, [32 ..] head (HR samples), then tail (HL samples)
#include <algorithm>
#include <string>

#include "fir_common.h"
#include "fir_launch.h"

namespace fir {

namespace {

constexpr uint32_t kGateLine = 32;  // dwords per 128-byte line

__host__ __device__ constexpr uint32_t gate_round_dw(int64_t bytes) {
    return (uint32_t)(((bytes + 127) / 128) * kGateLine);
}
__host__ __device__ constexpr uint32_t gate_slot_dw(int64_t hl_bytes, int64_t hr_bytes) {
    return kGateLine + gate_round_dw(hr_bytes) + gate_round_dw(hl_bytes);
}

// A read-modify-write that adds `zero` (a kernel argument the host sets to 0): a constant 0
// would let the compiler turn it into a plain system-scope load, which is served from the
// reading XCD's L2 (a stale line can stay there), whereas an RMW is performed at the memory side.
__device__ __forceinline__ uint32_t mb_read(const uint32_t* p, uint32_t zero) {
    return __hip_atomic_fetch_add(const_cast<uint32_t*>(p), zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t mb_write(uint32_t* p, uint32_t v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// dword i of the byte range [p, p + n): little-endian bytes, zero past n (byte loads: the
// ranges are a few samples and need not be dword aligned)
__device__ __forceinline__ uint32_t gather_dword(const uint8_t* p, int64_t n, int64_t i) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int64_t k = 4 * i + b;
        if (k < n) w |= (uint32_t)p[k] << (8 * b);
    }
    return w;
}
__device__ __forceinline__ void scatter_dword(uint8_t* p, int64_t n, int64_t i, uint32_t w) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int64_t k = 4 * i + b;
        if (k < n) p[k] = (uint8_t)(w >> (8 * b));
    }
}

// One wave.  Waits are done by lane 0 with s_sleep between polls (one poller per rank).
__global__ __launch_bounds__(kWave) void halo_gate_kernel(const uint8_t* __restrict__ x, int64_t seg_bytes,
                                                          int64_t hl_bytes, int64_t hr_bytes, uint32_t* own,
                                                          const uint32_t* left, const uint32_t* right,
                                                          uint8_t* __restrict__ out_l, uint8_t* __restrict__ out_r,
                                                          int32_t* __restrict__ status_out, uint64_t timeout_ticks,
                                                          uint32_t zero) {
    const int lane = threadIdx.x;
    const uint32_t slot_dw = gate_slot_dw(hl_bytes, hr_bytes);
    const uint32_t head0 = kGateLine, tail0 = kGateLine + gate_round_dw(hr_bytes);
    const int64_t hr_dw = (hr_bytes + 3) / 4, hl_dw = (hl_bytes + 3) / 4;

    // lane 0 reads the gate count and status (the same for every lane after the broadcast), and
    // checks that every mailbox this gate indexes is laid out for its halo sizes
    uint32_t cnt = 0, status = 0, layout_ok = 1;
    if (lane == 0) {
        const uint32_t* mbs[3] = {own, left, right};
        for (int m = 0; m < 3; ++m)
            if (mbs[m] && (mb_read(&mbs[m][2], zero) != (uint32_t)hl_bytes || mb_read(&mbs[m][3], zero) != (uint32_t)hr_bytes))
                layout_ok = 0;
        cnt = mb_read(&own[0], zero);
        status = mb_read(&own[1], zero);
    }
    layout_ok = __shfl(layout_ok, 0);
    if (!layout_ok) {  // no slot is touched; the halos are zeroed
        if (lane == 0 && status_out) *status_out = (int32_t)FIR_GATE_LAYOUT;
        for (int64_t i = lane; out_l && i < hl_bytes; i += kWave) out_l[i] = 0;
        for (int64_t i = lane; out_r && i < hr_bytes; i += kWave) out_r[i] = 0;
        return;
    }
    cnt = __shfl(cnt, 0);
    status = __shfl(status, 0);
    const uint32_t epoch = cnt + 1;
    const uint32_t s = 32 + (epoch & 1u) * slot_dw;

    // 1. publish this step's edges, then (after every payload atomic has completed) the epoch
    uint32_t sink = 0;
    for (int64_t i = lane; i < hr_dw; i += kWave) sink |= mb_write(&own[s + head0 + i], gather_dword(x, hr_bytes, i));
    const uint8_t* tail = x + (seg_bytes - hl_bytes);
    for (int64_t i = lane; i < hl_dw; i += kWave) sink |= mb_write(&own[s + tail0 + i], gather_dword(tail, hl_bytes, i));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        sink |= mb_write(&own[s], epoch);
        sink |= mb_write(&own[0], epoch);
    }

    // 2. wait for both neighbours' epoch (bounded)
    uint32_t ok = 1;
    if (lane == 0 && status == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
        const uint32_t* nbs[2] = {left, right};
        for (int j = 0; j < 2; ++j) {
            const uint32_t* nb = nbs[j];
            if (!nb) continue;
            while (mb_read(&nb[s], zero) != epoch) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (!ok) break;
        }
        if (!ok) sink |= mb_write(&own[1], (uint32_t)FIR_GATE_TIMEOUT);
    }
    ok = __shfl(ok, 0) && status == 0;
    if (lane == 0 && status_out) *status_out = ok ? 0 : (int32_t)FIR_GATE_TIMEOUT;  // plain, read by the host

    // 3. the neighbours' samples into the local halo buffers (zeros after a timeout)
    if (out_l) {
        for (int64_t i = lane; i < hl_dw; i += kWave)
            scatter_dword(out_l, hl_bytes, i, ok && left ? mb_read(&left[s + tail0 + i], zero) : 0u);
    }
    if (out_r) {
        for (int64_t i = lane; i < hr_dw; i += kWave)
            scatter_dword(out_r, hr_bytes, i, ok && right ? mb_read(&right[s + head0 + i], zero) : 0u);
    }
    // keep the returning atomics' results live (never true: seg_bytes >= 0 is checked on the host)
    if (sink == 0x9E3779B9u && seg_bytes < 0 && status_out) *status_out = (int32_t)sink;
}

__global__ __launch_bounds__(kBlock) void halo_mailbox_init_kernel(uint32_t* mb, int64_t ndw, uint32_t hl_bytes,
                                                                   uint32_t hr_bytes) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < ndw; i += (int64_t)gridDim.x * kBlock)
        (void)mb_write(&mb[i], i == 2 ? hl_bytes : i == 3 ? hr_bytes : 0u);
}

}  // namespace

int64_t halo_mailbox_bytes(int64_t hl_bytes, int64_t hr_bytes) {
    return 4 * (32 + 2 * (int64_t)gate_slot_dw(hl_bytes, hr_bytes));
}

int launch_halo_mailbox_init(void* mailbox, int64_t bytes, int64_t hl_bytes, int64_t hr_bytes, hipStream_t stream,
                             std::string* err) {
    if (hl_bytes < 0 || hr_bytes < 0 || hl_bytes >= (1ll << 31) || hr_bytes >= (1ll << 31))
        return *err = "halo byte counts must be in [0, 2^31)", FIR_EINVAL;
    if (!mailbox || bytes < halo_mailbox_bytes(hl_bytes, hr_bytes) || bytes % 4)
        return *err = "mailbox must hold fir_halo_mailbox_bytes(halo sizes) bytes, a multiple of 4", FIR_EINVAL;
    if ((uintptr_t)mailbox % 128) return *err = "mailbox must be 128-byte aligned", FIR_EINVAL;
    const int64_t ndw = bytes / 4;
    const int64_t blocks = std::min<int64_t>((ndw + kBlock - 1) / kBlock, 1024);
    hipLaunchKernelGGL(halo_mailbox_init_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, (uint32_t*)mailbox, ndw,
                       (uint32_t)hl_bytes, (uint32_t)hr_bytes);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("halo mailbox init launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

int launch_halo_gate(const void* x, int64_t seg_bytes, int64_t hl_bytes, int64_t hr_bytes, void* mailbox,
                     const void* left_mailbox, const void* right_mailbox, void* halo_left, void* halo_right,
                     int32_t* status, double timeout_s, hipStream_t stream, std::string* err) {
    if (hl_bytes < 0 || hr_bytes < 0 || seg_bytes < hl_bytes || seg_bytes < hr_bytes || hl_bytes >= (1ll << 31) ||
        hr_bytes >= (1ll << 31))
        return *err = "halo byte counts must be in [0, min(seg_bytes, 2^31 - 1)]", FIR_EINVAL;
    if (!mailbox) return *err = "mailbox must not be NULL", FIR_EINVAL;
    if ((!x && (hl_bytes || hr_bytes)) || (left_mailbox && hl_bytes && !halo_left) ||
        (right_mailbox && hr_bytes && !halo_right))
        return *err = "x and the halo buffers of present neighbours must not be NULL", FIR_EINVAL;
    if ((uintptr_t)mailbox % 128 || (uintptr_t)left_mailbox % 128 || (uintptr_t)right_mailbox % 128)
        return *err = "mailboxes must be 128-byte aligned", FIR_EINVAL;
    if (!(timeout_s > 0.0) || timeout_s > 600.0) return *err = "timeout_s must be in (0, 600]", FIR_EINVAL;
    const uint64_t ticks = (uint64_t)(timeout_s * 1e8);  // s_memrealtime runs at 100 MHz
    hipLaunchKernelGGL(halo_gate_kernel, dim3(1), dim3(kWave), 0, stream, (const uint8_t*)x, seg_bytes, hl_bytes,
                       hr_bytes, (uint32_t*)mailbox, (const uint32_t*)left_mailbox, (const uint32_t*)right_mailbox,
                       left_mailbox ? (uint8_t*)halo_left : nullptr, right_mailbox ? (uint8_t*)halo_right : nullptr,
                       status, ticks, 0u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return *err = std::string("halo gate launch failed: ") + hipGetErrorString(e), FIR_EHIP;
    return FIR_OK;
}

}  // namespace fir

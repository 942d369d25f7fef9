// dev_tables.hip — device copies of host-side tables (long tap sets, matrix-core tap fragments).
//
// Short filters travel in the kernel arguments; a filter of any length (the reference accepts
// any len(h), fir_1d/model/python/fir_1d_fixed_ref.py:83-107) does not fit there, so its taps
// are read from HBM.  The C ABI keeps taking host pointers; this cache uploads each distinct
// table once per device and hands out its device address.
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "fir_launch.h"

namespace fir {

namespace {

constexpr size_t kTableBudget = size_t(256) << 20;  // bytes cached per device before a flush

struct TableCache {
    std::mutex mu;
    hipStream_t stream = nullptr;
    std::map<std::string, void*> tables;  // content -> device copy
    size_t bytes = 0;
};

std::mutex g_caches_mu;
std::map<int, std::unique_ptr<TableCache>> g_caches;

TableCache* cache_for(int dev) {
    std::lock_guard<std::mutex> lk(g_caches_mu);
    auto& c = g_caches[dev];
    if (!c) c.reset(new TableCache());
    return c.get();
}

}  // namespace

const void* device_table(const void* host, size_t bytes, std::string* err) {
    if (!host || bytes == 0) {
        *err = "device_table: empty table";
        return nullptr;
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        *err = std::string("hipGetDevice: ") + hipGetErrorString(e);
        return nullptr;
    }
    TableCache* c = cache_for(dev);
    std::string key((const char*)host, bytes);
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->tables.find(key);
    if (it != c->tables.end()) return it->second;
    if (!c->stream && (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
        *err = std::string("hipStreamCreateWithFlags: ") + hipGetErrorString(e);
        return nullptr;
    }
    if (c->bytes + bytes > kTableBudget && !c->tables.empty()) {
        // every launch that may still read a cached table must have finished before it is freed
        if ((e = hipDeviceSynchronize()) != hipSuccess) {
            *err = std::string("hipDeviceSynchronize: ") + hipGetErrorString(e);
            return nullptr;
        }
        for (auto& kv : c->tables) (void)hipFree(kv.second);
        c->tables.clear();
        c->bytes = 0;
    }
    void* d = nullptr;
    if ((e = hipMalloc(&d, bytes)) != hipSuccess) {
        *err = std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e);
        return nullptr;
    }
    // complete before this returns, so any later launch on any stream sees the whole table
    if ((e = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        (void)hipFree(d);
        *err = std::string("table upload: ") + hipGetErrorString(e);
        return nullptr;
    }
    c->tables.emplace(std::move(key), d);
    c->bytes += bytes;
    return d;
}

}  // namespace fir

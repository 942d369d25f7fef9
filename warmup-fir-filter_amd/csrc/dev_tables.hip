// dev_tables.hip — device copies of host-side tables (long tap sets, matrix-core tap fragments).
//
// Short filters travel in the kernel arguments; a filter of any length (the reference accepts
// any len(h), fir_1d/model/python/fir_1d_fixed_ref.py:83-107) does not fit there, so its taps
// are read from HBM.  The C ABI keeps taking host pointers; this cache uploads each distinct
// table once per device and hands out its device address for one launch at a time (TableHold):
//
//   * a table is keyed by the bytes it is made from (its content, or the inputs a large derived
//     table is built from, so that one is built only on a miss) behind a kind tag: looked up by a
//     128-bit hash and its size, confirmed by comparing those bytes (a collision is a miss);
//   * every hold counts as in use until the launch it was taken for has been enqueued, and each
//     use then records an event of its own behind that launch, kept until it has completed
//     (completed ones go back to a pool, oldest first, so the events held stay bounded by the
//     launches in flight).  No event is ever re-recorded while its record is pending: that would
//     assume the stream handle still names the stream that made the record, and a destroyed
//     stream's handle may be handed to a new stream while the old one's launches still run
//     (hipStreamDestroy may return with work in flight).  A table is freed only when it has no
//     hold and every use's event has completed, never by a device-wide sync (which would also
//     invalidate another thread's stream capture);
//   * a table used by a launch that was captured into a hipGraph is pinned for the process life
//     (the graph keeps its address);
//   * past kTableBudget bytes per device the cache frees idle tables; when none is idle it grows
//     past the budget rather than fail a call.
#include <hip/hip_runtime.h>

#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "fir_launch.h"

namespace fir {

namespace {

constexpr size_t kTableBudget = size_t(256) << 20;  // idle bytes kept per device

struct Entry {
    void* d = nullptr;
    size_t bytes = 0;
    int holds = 0;                  // acquired, launch not yet enqueued
    bool pinned = false;            // used by a captured graph
    // one event per use whose completion has not been seen yet, in record order
    std::deque<hipEvent_t> uses;
};

// (hash, size) first: the source bytes are compared only between tables whose hashes are equal
using Key = std::tuple<uint64_t, uint64_t, size_t, std::vector<uint8_t>>;
using TableMap = std::map<Key, Entry>;

struct TableCache {
    std::mutex mu;
    hipStream_t stream = nullptr;
    TableMap tables;
    std::map<const void*, TableMap::iterator> by_ptr;
    std::vector<hipEvent_t> free_events;
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

// return the completed events at the front of e's uses to the pool (oldest first: amortised
// O(1) per use; a completed event behind a pending one waits for that one)
void prune(TableCache* c, Entry& e) {
    while (!e.uses.empty() && hipEventQuery(e.uses.front()) == hipSuccess) {
        c->free_events.push_back(e.uses.front());
        e.uses.pop_front();
    }
}

// true when every recorded use of e has completed (completed events go back to the pool)
bool idle(TableCache* c, Entry& e) {
    std::deque<hipEvent_t> pending;
    for (hipEvent_t ev : e.uses) {
        if (hipEventQuery(ev) == hipSuccess) c->free_events.push_back(ev);
        else pending.push_back(ev);
    }
    e.uses.swap(pending);
    return e.holds == 0 && !e.pinned && e.uses.empty();
}

void evict_idle(TableCache* c, size_t need) {
    for (auto it = c->tables.begin(); it != c->tables.end() && c->bytes + need > kTableBudget;) {
        if (idle(c, it->second)) {
            (void)hipFree(it->second.d);
            c->bytes -= it->second.bytes;
            c->by_ptr.erase(it->second.d);
            it = c->tables.erase(it);
        } else {
            ++it;
        }
    }
}

}  // namespace

void TableHash::add(const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    src.insert(src.end(), b, b + n);
    for (size_t i = 0; i < n; ++i) {
        a = (a ^ b[i]) * 0x100000001b3ull;                          // FNV-1a 64
        c = (c + b[i] + 0x9E3779B97F4A7C15ull) * 0xff51afd7ed558ccdull;  // an independent mix
        c ^= c >> 29;
    }
}

const void* table_acquire(TableHash&& h, size_t bytes, const std::function<void(void*)>& fill, std::string* err) {
    if (bytes == 0) {
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
    Key key{h.a, h.c, bytes, std::move(h.src)};  // the identity bytes move, once: no copy on a hit
    std::lock_guard<std::mutex> lk(c->mu);
    auto it = c->tables.find(key);
    if (it != c->tables.end()) {
        ++it->second.holds;
        return it->second.d;
    }
    if (!c->stream && (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
        *err = std::string("hipStreamCreateWithFlags: ") + hipGetErrorString(e);
        return nullptr;
    }
    evict_idle(c, bytes);
    std::vector<uint8_t> host(bytes);
    fill(host.data());
    void* d = nullptr;
    if ((e = hipMalloc(&d, bytes)) != hipSuccess) {
        *err = std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e);
        return nullptr;
    }
    // complete before this returns, so any later launch on any stream sees the whole table
    if ((e = hipMemcpyAsync(d, host.data(), bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        (void)hipFree(d);
        *err = std::string("table upload: ") + hipGetErrorString(e);
        return nullptr;
    }
    const auto ins = c->tables.emplace(std::move(key), Entry{}).first;
    Entry& en = ins->second;
    en.d = d;
    en.bytes = bytes;
    en.holds = 1;
    c->by_ptr[d] = ins;
    c->bytes += bytes;
    return d;
}

void table_release(const void* d, hipStream_t stream, bool launched) {
    if (!d) return;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    TableCache* c = cache_for(dev);
    std::lock_guard<std::mutex> lk(c->mu);
    auto pit = c->by_ptr.find(d);
    if (pit == c->by_ptr.end()) return;
    Entry& en = pit->second->second;
    if (en.holds > 0) --en.holds;
    if (!launched) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        en.pinned = true;  // a graph holds the address for as long as it lives
        return;
    }
    prune(c, en);
    hipEvent_t ev = nullptr;
    if (!c->free_events.empty()) {
        ev = c->free_events.back();
        c->free_events.pop_back();
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        en.pinned = true;  // cannot track the use: never free it
        return;
    }
    if (hipEventRecord(ev, stream) != hipSuccess) {
        c->free_events.push_back(ev);
        en.pinned = true;
        return;
    }
    en.uses.push_back(ev);
}

const void* device_table(const void* host, size_t bytes, std::string* err) {
    if (!host) {
        *err = "device_table: empty table";
        return nullptr;
    }
    TableHash h(kTableRaw);
    h.add(host, bytes);
    return table_acquire(std::move(h), bytes, [&](void* dst) { std::memcpy(dst, host, bytes); }, err);
}

}  // namespace fir

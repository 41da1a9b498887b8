// Host-only bookkeeping of a context's verify workspaces and of its concurrency slots
// (cc_set_concurrency, capi.cpp): the bytes a batch of n credentials needs in each workspace, the
// workspace set one launch reads (every member named), the round-robin choice of a slot, and the
// protocol that keeps a slot's buffers alive while its last batch may still read them:
//
//   begin  the next slot: if one of its workspaces is short, the host waits for the slot's last batch
//          (its `done` event) BEFORE the buffer is reallocated; the launch stream is then ordered after
//          the context stream's queued work and after that last batch;
//   end    records the slot's `done` on the launch stream;
//   Fence  (RAII) ends a begun slot on every exit, so a launch that fails half-way still fences the
//          kernels it queued (the next user of the slot waits for them before growing the buffers).
//
// No HIP types here: the device is a policy class.  capi.cpp instantiates it over hipMalloc'd buffers
// and hipEvent_t (HipDev); tests/host/test_slots.cpp over a simulated device timeline that flags a
// buffer reallocated while a queued operation still reads it, built with -fsanitize=address,undefined
// (tests/test_host_slots.py, `pytest -m "not gpu"`).
#pragma once
#include <stddef.h>

#include <vector>

namespace cc {
namespace slots {

constexpr size_t kPrepSlots = 14;  // Fp slots of the prep SoA (soa.h)
// Small batches run the one-wave kernels (capi.cpp launch_miller / launch_verify): the Miller loop one
// wave per pair up to kWideMax credentials (its own prep / flags / Miller-value workspaces), the final
// exponentiation one wave per credential up to kFexpWideMax (its chain in the scratch), the PoK and
// per-credential-verkey preps one wave per credential up to kPrepWideMax.
constexpr size_t kWideMax = 4096;
constexpr size_t kFexpWideMax = 2048;
constexpr size_t kPrepWideMax = 1024;

// bytes per workspace for one batch
struct Sizes {
    size_t prep = 0, flags = 0, fbuf = 0, vkb = 0, scratch = 0, idx = 0, wprep = 0, wflags = 0, wf = 0;
    size_t at(int k) const {
        const size_t a[] = {prep, flags, fbuf, vkb, scratch, idx, wprep, wflags, wf};
        return a[k];
    }
};

// n credentials; vkw: per-credential-verkey MSM scratch (0: shared verkey); scratch_bytes: the PoK's
// tables of d J; idx_bytes: the PoK's revealed indices
inline Sizes verify_sizes(size_t n, size_t vkw, size_t scratch_bytes, size_t idx_bytes) {
    Sizes s;
    const size_t words = n * 12;  // one Fp slot
    s.prep = words * 4 * kPrepSlots;
    s.flags = n * 4;
    s.fbuf = words * 4 * 12;
    s.vkb = vkw;
    s.scratch = scratch_bytes;
    if (n <= kFexpWideMax && s.scratch < 72 * 12 * n * 4) s.scratch = 72 * 12 * n * 4;  // k_fexp1's chain
    s.idx = idx_bytes;
    if (n <= kWideMax) {  // one wave per pair: 2 n pairs
        const size_t m = 2 * n;
        s.wprep = m * 12 * 4 * kPrepSlots;
        s.wflags = m * 4;
        s.wf = m * 12 * 4 * 12;
    }
    return s;
}

// The workspaces one verify / PoK launch reads.  Every member is named by the one constructor, so a
// partial list does not compile; complete() is checked again before a slot is used (a null member
// would be a null device pointer in a kernel argument).
template <class Buf>
struct Work {
    static constexpr int kN = 9;
    Buf *prep = nullptr, *flags = nullptr, *fbuf = nullptr, *vkb = nullptr, *scratch = nullptr, *idx = nullptr;
    Buf *wprep = nullptr, *wflags = nullptr, *wf = nullptr;  // the small-batch Miller path's
    Work() = default;
    Work(Buf* p, Buf* f, Buf* fb, Buf* v, Buf* s, Buf* i, Buf* wp, Buf* wfl, Buf* wv)
        : prep(p), flags(f), fbuf(fb), vkb(v), scratch(s), idx(i), wprep(wp), wflags(wfl), wf(wv) {}
    Buf* at(int k) const {
        Buf* const a[] = {prep, flags, fbuf, vkb, scratch, idx, wprep, wflags, wf};
        return a[k];
    }
    bool complete() const {
        for (int k = 0; k < kN; k++)
            if (!at(k)) return false;
        return true;
    }
    // some workspace is smaller than the batch needs
    bool short_of(const Sizes& s) const {
        for (int k = 0; k < kN; k++)
            if (at(k)->bytes < s.at(k)) return true;
        return false;
    }
};

// A concurrency slot's own buffers (slots 1 .. K-1; slot 0 is the context's workspaces): the verify
// workspaces and the RLC partial's (delta key, fall-back flag, fold points, digits, fold workspace).
template <class Buf>
struct SlotBufs {
    Buf prep, flags, fbuf, vkb, scratch, idx, wprep, wflags, wf;
    Buf rkey, rany, rpts, rdig, rwork;
    Work<Buf> work() { return Work<Buf>(&prep, &flags, &fbuf, &vkb, &scratch, &idx, &wprep, &wflags, &wf); }
    template <class F>
    void each(F f) {
        for (Buf* b : {&prep, &flags, &fbuf, &vkb, &scratch, &idx, &wprep, &wflags, &wf, &rkey, &rany, &rpts, &rdig, &rwork})
            f(*b);
    }
};

// The slots of one context.  Dev provides Buf (with .bytes), Event, Stream and
//   int ensure(Buf&, size_t)   grow to at least n bytes (0 ok)
//   int sync(Event)            host waits for the event
//   int record(Event, Stream)  event marks the stream's queued work
//   int wait(Stream, Event)    stream waits (on the device) for the event
template <class Dev>
struct Pool {
    using Buf = typename Dev::Buf;
    using Event = typename Dev::Event;
    using Stream = typename Dev::Stream;
    struct Rec {
        Work<Buf> w;
        Event done{};
        bool recorded = false;
    };
    std::vector<Rec> recs;  // recs[0]: the context's own workspaces
    int next = 0;

    int size() const { return (int)recs.size(); }
    // the next slot, round-robin
    int take() {
        const int k = next;
        next = (next + 1) % (int)recs.size();
        return k;
    }
    // slot k takes a batch of sizes s on stream st: grow its workspaces (after its last batch ended),
    // then order st after the context stream (ctx, through order_ev) and after the slot's last batch.
    // -2: the slot's workspace set is incomplete; -1: device error.
    int begin(Dev& d, int k, const Sizes& s, Stream st, Stream ctx, Event order_ev) {
        Rec& r = recs[(size_t)k];
        if (!r.w.complete()) return -2;
        if (r.w.short_of(s)) {
            if (r.recorded && d.sync(r.done)) return -1;  // its last batch still reads the buffers
            for (int j = 0; j < Work<Buf>::kN; j++)
                if (d.ensure(*r.w.at(j), s.at(j))) return -1;
        }
        if (st != ctx) {
            if (d.record(order_ev, ctx) || d.wait(st, order_ev)) return -1;
        }
        if (r.recorded && d.wait(st, r.done)) return -1;
        return 0;
    }
    int end(Dev& d, int k, Stream st) {
        Rec& r = recs[(size_t)k];
        if (d.record(r.done, st)) return -1;
        r.recorded = true;
        return 0;
    }
    // the host waits for every slot's last batch (before shared buffers are freed or rebuilt)
    void drain(Dev& d) {
        for (Rec& r : recs)
            if (r.recorded) (void)d.sync(r.done);
    }
    // stream st waits (on the device) for every slot's last batch
    void wait_all(Dev& d, Stream st) {
        for (Rec& r : recs)
            if (r.recorded) (void)d.wait(st, r.done);
    }
};

// Ends a begun slot on every exit: a launch that fails after queueing some kernels still records the
// slot's done event behind them.
template <class Dev>
struct Fence {
    Pool<Dev>& pool;
    Dev& dev;
    int k;
    typename Dev::Stream st;
    bool armed = true;
    Fence(Pool<Dev>& p, Dev& d, int slot, typename Dev::Stream s) : pool(p), dev(d), k(slot), st(s) {}
    // the normal exit: end the slot and report its status
    int close() {
        armed = false;
        return pool.end(dev, k, st);
    }
    ~Fence() {
        if (armed) (void)pool.end(dev, k, st);
    }
    Fence(const Fence&) = delete;
    Fence& operator=(const Fence&) = delete;
};

}  // namespace slots
}  // namespace cc

// Host-only test of the concurrency-slot bookkeeping (coconut-rust_amd/csrc/slots.h) that capi.cpp
// runs over HIP.  Here the device is simulated: every stream is a FIFO of queued operations, an event
// marks a stream position, a "kernel" reads a set of buffers (id + allocation generation), and a buffer
// reallocated while a queued operation still reads its old allocation is counted as a use-after-free
// (what the GPU would do with a hipFree'd workspace).  Built with -fsanitize=address,undefined by
// tests/test_sanitizers.py; exits non-zero on the first failed check.
#include <stdio.h>
#include <stdlib.h>

#include <deque>
#include <map>
#include <vector>

#include "slots.h"

using namespace cc::slots;

static int g_fail = 0;
#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                    \
        }                                                                \
    } while (0)

struct FakeBuf {
    int id = 0;
    size_t bytes = 0;
    int gen = 0;
};

struct FakeDev {
    using Buf = FakeBuf;
    using Event = int;   // index into evs (0: not created)
    using Stream = int;  // index into streams
    struct Op {
        long seq;
        std::vector<std::pair<int, int>> reads;  // (buffer id, generation)
        int wait_stream = -1;                    // a wait: completes after that stream reaches wait_seq
        long wait_seq = -1;
    };
    std::vector<std::deque<Op>> streams;
    std::map<int, std::pair<int, long>> evs;  // event -> (stream, seq of its last op when recorded)
    long seq = 0;
    int next_buf = 1, next_ev = 1;
    int uaf = 0;       // reallocations under a queued reader
    int bad_read = 0;  // kernels launched on a null / undersized workspace

    explicit FakeDev(int nstreams) : streams((size_t)nstreams) {}
    Event new_event() { return next_ev++; }
    void name(FakeBuf& b) {
        if (!b.id) b.id = next_buf++;
    }
    bool read_pending(int id, int gen) const {
        for (const auto& q : streams)
            for (const Op& o : q)
                for (auto& r : o.reads)
                    if (r.first == id && r.second == gen) return true;
        return false;
    }
    // --- the policy slots.h needs
    int ensure(FakeBuf& b, size_t n) {
        name(b);
        if (n <= b.bytes) return 0;
        if (b.bytes && read_pending(b.id, b.gen)) uaf++;
        b.gen++;
        b.bytes = n;
        return 0;
    }
    int record(Event e, Stream s) {
        if (!e) return -1;
        evs[e] = {s, streams[(size_t)s].empty() ? -1 : streams[(size_t)s].back().seq};
        return 0;
    }
    int wait(Stream s, Event e) {
        auto it = evs.find(e);
        if (it == evs.end()) return 0;  // never recorded: nothing to wait for
        Op o;
        o.seq = ++seq;
        o.wait_stream = it->second.first;
        o.wait_seq = it->second.second;
        streams[(size_t)s].push_back(o);
        return 0;
    }
    int sync(Event e) {
        auto it = evs.find(e);
        if (it == evs.end()) return 0;
        run_until(it->second.first, it->second.second);
        return 0;
    }
    // --- the simulated device
    // completes stream s's operations up to seq (waits first complete what they wait for)
    void run_until(int s, long upto) {
        auto& q = streams[(size_t)s];
        while (!q.empty() && q.front().seq <= upto) {
            Op o = q.front();
            if (o.wait_stream >= 0) run_until(o.wait_stream, o.wait_seq);
            q.pop_front();
        }
    }
    void run_all() {
        for (size_t s = 0; s < streams.size(); s++) run_until((int)s, seq);
    }
    // a kernel on stream s reading the workspaces w needs for sizes sz
    void launch(Stream s, const Work<FakeBuf>& w, const Sizes& sz) {
        Op o;
        o.seq = ++seq;
        for (int k = 0; k < Work<FakeBuf>::kN; k++) {
            FakeBuf* b = w.at(k);
            if (!b || b->bytes < sz.at(k)) {
                bad_read++;
                continue;
            }
            if (sz.at(k)) o.reads.push_back({b->id, b->gen});
        }
        streams[(size_t)s].push_back(o);
    }
};

// a context's slot 0 (its own workspaces) + K-1 slot buffer sets, as capi.cpp cc_set_concurrency builds
struct Ctx {
    FakeDev dev;
    Pool<FakeDev> pool;
    SlotBufs<FakeBuf> own;
    std::vector<SlotBufs<FakeBuf>*> extra;
    FakeDev::Event order_ev;
    static constexpr int kCtxStream = 0;
    Ctx(int K, int nstreams) : dev(nstreams) {
        order_ev = dev.new_event();
        pool.recs.resize((size_t)K);
        pool.recs[0].w = own.work();
        pool.recs[0].done = dev.new_event();
        for (int k = 1; k < K; k++) {
            extra.push_back(new SlotBufs<FakeBuf>);
            pool.recs[(size_t)k].w = extra.back()->work();
            pool.recs[(size_t)k].done = dev.new_event();
        }
    }
    ~Ctx() {
        for (auto* e : extra) delete e;
    }
    // one verify batch as capi.cpp verify_device runs it on a slot; fail_after: the launch "fails" after
    // queueing that many kernels (the Fence must still end the slot)
    int batch(int stream, size_t n, size_t vkw = 0, int fail_after = -1, bool use_fence = true) {
        const Sizes sz = verify_sizes(n, vkw, 0, 0);
        const int k = pool.take();
        const int rc = pool.begin(dev, k, sz, stream, kCtxStream, order_ev);
        if (rc) return rc;
        if (!use_fence) {  // the pre-Fence code path: a failed launch returned without recording done
            for (int j = 0; j < 3; j++) {
                if (j == fail_after) return -7;
                dev.launch(stream, pool.recs[(size_t)k].w, sz);
            }
            return pool.end(dev, k, stream);
        }
        Fence<FakeDev> fence(pool, dev, k, stream);
        for (int j = 0; j < 3; j++) {  // prep, Miller, fexp
            if (j == fail_after) return -7;
            dev.launch(stream, pool.recs[(size_t)k].w, sz);
        }
        return fence.close();
    }
};

static void test_sizes() {
    const Sizes a = verify_sizes(100, 0, 0, 0);
    CHECK(a.prep == 100 * 12 * 4 * kPrepSlots && a.flags == 400 && a.fbuf == 100 * 12 * 4 * 12);
    CHECK(a.scratch == 72 * 12 * 100 * 4);  // k_fexp1's chain below kFexpWideMax
    CHECK(a.wprep == 200 * 12 * 4 * kPrepSlots && a.wflags == 800 && a.wf == 200 * 12 * 4 * 12);
    const Sizes b = verify_sizes(kWideMax + 1, 123, 0, 8);
    CHECK(b.scratch == 0 && b.wprep == 0 && b.wflags == 0 && b.wf == 0 && b.vkb == 123 && b.idx == 8);
    const Sizes c = verify_sizes(kFexpWideMax + 1, 0, 0, 0);
    CHECK(c.scratch == 0 && c.wprep > 0);  // the wide Miller path reaches further than the wide fexp
}

static void test_work_complete() {
    SlotBufs<FakeBuf> s;
    Work<FakeBuf> w = s.work();
    CHECK(w.complete());
    for (int k = 0; k < Work<FakeBuf>::kN; k++) {
        Work<FakeBuf> v = w;
        // knock out workspace k (what round 5's partial aggregate did for scratch / idx)
        FakeBuf** m[] = {&v.prep, &v.flags, &v.fbuf, &v.vkb, &v.scratch, &v.idx, &v.wprep, &v.wflags, &v.wf};
        *m[k] = nullptr;
        CHECK(!v.complete());
        // a pool slot holding it refuses the batch instead of launching on a null workspace
        FakeDev dev(2);
        Pool<FakeDev> p;
        p.recs.resize(1);
        p.recs[0].w = v;
        p.recs[0].done = dev.new_event();
        CHECK(p.begin(dev, 0, verify_sizes(16, 0, 0, 0), 1, 0, dev.new_event()) == -2);
        CHECK(dev.bad_read == 0);
    }
    Work<FakeBuf> d;  // default-constructed: nothing named
    CHECK(!d.complete());
}

static void test_round_robin() {
    Ctx c(3, 4);
    int seen[3] = {0, 0, 0};
    for (int j = 0; j < 9; j++) seen[c.pool.take()]++;
    CHECK(seen[0] == 3 && seen[1] == 3 && seen[2] == 3);
}

// K = 2, batches alternating on two streams; the third batch lands on slot 0 again and is larger: the
// pool must wait for slot 0's first batch before it grows the buffers that batch still reads
static void test_reuse_waits_for_inflight() {
    Ctx c(2, 3);
    CHECK(c.batch(1, 1000) == 0);  // slot 0
    CHECK(c.batch(2, 1000) == 0);  // slot 1
    CHECK(c.dev.uaf == 0);
    CHECK(c.batch(1, 5000) == 0);  // slot 0, grows: waits for batch 1 first
    CHECK(c.batch(2, 8000, 4096) == 0);  // slot 1, grows (and a per-verkey scratch)
    CHECK(c.dev.uaf == 0 && c.dev.bad_read == 0);
    // same-size reuse: no growth, the stream waits on the device instead (no host wait, no realloc)
    const int gen0 = c.own.prep.gen;
    CHECK(c.batch(1, 5000) == 0);
    CHECK(c.own.prep.gen == gen0 && c.dev.uaf == 0);
    c.dev.run_all();
}

// the simulated device does flag the bug class: growing a slot's buffer with its batch still queued
static void test_detector_has_teeth() {
    Ctx c(2, 3);
    CHECK(c.batch(1, 1000) == 0);
    c.dev.ensure(c.own.prep, 1u << 30);  // reallocation without waiting for the slot's batch
    CHECK(c.dev.uaf == 1);
}

// a launch failing half-way: the Fence still records the slot's done behind the kernels it queued, so
// the next (larger) batch on that slot waits for them
static void test_fence_on_failure() {
    Ctx c(2, 3);
    CHECK(c.batch(1, 1000, 0, /*fail_after=*/2) == -7);
    CHECK(c.batch(2, 1000) == 0);
    CHECK(c.batch(1, 9000) == 0);
    CHECK(c.dev.uaf == 0);
    // without the fence (the pre-round-6 path) the same sequence reallocates under a queued kernel
    Ctx d(2, 3);
    CHECK(d.batch(1, 1000) == 0);
    CHECK(d.batch(2, 1000) == 0);
    CHECK(d.batch(1, 1000, 0, 2, /*use_fence=*/false) == -7);  // slot 0: kernels queued, done not recorded
    CHECK(d.batch(2, 1000) == 0);
    CHECK(d.batch(1, 9000) == 0);  // slot 0 grows, but its done marks the batch before the failed one
    CHECK(d.dev.uaf > 0);
}

// drain waits for every slot; wait_all orders a stream after every slot's last batch
static void test_drain() {
    Ctx c(3, 4);
    CHECK(c.batch(1, 500) == 0);
    CHECK(c.batch(2, 500) == 0);
    CHECK(c.batch(3, 500) == 0);
    c.pool.drain(c.dev);
    for (auto& q : c.dev.streams) CHECK(q.empty());
    // shared buffers (tables) may now be rebuilt: nothing queued reads anything
    CHECK(!c.dev.read_pending(c.own.prep.id, c.own.prep.gen));
}

int main() {
    test_sizes();
    test_work_complete();
    test_round_robin();
    test_reuse_waits_for_inflight();
    test_detector_has_teeth();
    test_fence_on_failure();
    test_drain();
    if (g_fail) {
        fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    printf("slots: all checks passed\n");
    return 0;
}

// C-ABI of the engine (include/thetarrt.h): context, device tree mirror, batch entry points,
// host bookkeeping (the reference's dict G / cameFrom, rrt.py:134-138,179-188) and the RRT session.
#include <string.h>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include <algorithm>
#include <vector>
#include <memory>
#include <new>
#include <string>
#include <math.h>
#include <vector>

#include "thetarrt_internal.hpp"

using namespace tr;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(TR_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define GUARD(...)                                                           \
  try {                                                                      \
    __VA_ARGS__                                                              \
  } catch (const std::bad_alloc&) {                                          \
    return fail(TR_E_HIP, "host allocation failed");                         \
  } catch (const std::exception& ex) {                                       \
    return fail(TR_E_HIP, ex.what());                                        \
  }

// Message of a device bookkeeping error (TR_DDE_* bits).
static std::string dde_message(int32_t bits) {
  if (bits & TR_DDE_GATE)
    return "device pipeline: a stream gate timed out waiting for the other stream (bits " +
           std::to_string(bits) + ")";
  return "device bookkeeping: a hash probe ran through a full table (bits " + std::to_string(bits) + ")";
}

// ------------------------------------------------------------------ device buffers
template <typename T>
struct DBuf {
  T* p = nullptr;
  int64_t cap = 0;
  hipError_t reserve(int64_t n) {
    if (n <= cap) return hipSuccess;
    int64_t c = std::max<int64_t>(n, cap * 2);
    T* q = nullptr;
    hipError_t e = hipMalloc(&q, sizeof(T) * (size_t)std::max<int64_t>(c, 1));
    if (e != hipSuccess) return e;
    if (p) (void)hipFree(p);
    p = q;
    cap = c;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <typename T>
struct HBuf {  // pinned host staging; flags = hipHostMalloc* (coherent = device writes bypass L2)
  T* p = nullptr;
  int64_t cap = 0;
  unsigned flags = 0;
  hipError_t reserve(int64_t n) {
    if (n <= cap) return hipSuccess;
    int64_t c = std::max<int64_t>(n, cap * 2);
    T* q = nullptr;
    hipError_t e = hipHostMalloc((void**)&q, sizeof(T) * (size_t)std::max<int64_t>(c, 1), flags);
    if (e != hipSuccess) return e;
    if (p) (void)hipHostFree(p);
    p = q;
    cap = c;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// hipMemset / device-to-device hipMemcpy run on the legacy null stream and do not wait for their
// work to finish, and the engine's streams are non-blocking (not ordered against the null stream):
// a kernel on st could run before such a clear.  Every fill and device copy of the engine goes on
// a given stream and is waited for.
static hipError_t fill_sync(hipStream_t st, void* p, int v, size_t n) {
  hipError_t e = hipMemsetAsync(p, v, n, st);
  return e != hipSuccess ? e : hipStreamSynchronize(st);
}
static hipError_t copy_sync(hipStream_t st, void* dst, const void* src, size_t n, hipMemcpyKind k) {
  hipError_t e = hipMemcpyAsync(dst, src, n, k, st);
  return e != hipSuccess ? e : hipStreamSynchronize(st);
}

// ------------------------------------------------------------------ host bookkeeping
static inline uint64_t dbits(double v) {
  if (v == 0.0) v = 0.0;  // Python: -0.0 == 0.0 and hash(-0.0) == hash(0.0)
  uint64_t b;
  memcpy(&b, &v, 8);
  return b;
}

static inline uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}

static inline uint64_t key_hash(double x, double y, double t) {
  return mix64(dbits(x) ^ mix64(dbits(y) + 0x9E3779B97F4A7C15ull) ^ mix64(dbits(t) + 0x632BE59BD9B4E019ull));
}

// Open-addressing index: exact-value pose -> node index (the reference's dict key test,
// rrt.py:151,179).  Keys live in the book's xyt array; slots hold (hash, index).
struct PoseIndex {
  struct Slot { uint64_t h; int64_t i; };
  std::vector<Slot> slots;
  uint64_t mask = 0;
  int64_t count = 0;

  void clear() {
    slots.assign(1024, Slot{0, -1});
    mask = 1023;
    count = 0;
  }
  template <typename Eq>
  int64_t find(uint64_t h, Eq eq) const {
    for (uint64_t p = h & mask;; p = (p + 1) & mask) {
      const Slot& s = slots[p];
      if (s.i < 0) return -1;
      if (s.h == h && eq(s.i)) return s.i;
    }
  }
  void insert(uint64_t h, int64_t i) {
    if (2 * (count + 1) > (int64_t)slots.size()) grow();
    uint64_t p = h & mask;
    while (slots[p].i >= 0) p = (p + 1) & mask;
    slots[p] = Slot{h, i};
    ++count;
  }
  void grow() {
    std::vector<Slot> old;
    old.swap(slots);
    slots.assign(old.size() * 2, Slot{0, -1});
    mask = slots.size() - 1;
    for (const Slot& s : old)
      if (s.i >= 0) {
        uint64_t p = s.h & mask;
        while (slots[p].i >= 0) p = (p + 1) & mask;
        slots[p] = s;
      }
  }
};

// Reserve and pre-fault: fresh pages would otherwise be faulted in one by one by the appends
// (measured: ~60 ns per appended node, all of it first-touch page faults).
// The book's arrays: resize() without a value leaves new elements uninitialised (the replay
// writes every one of them right away; zero-filling them first was a quarter of its time).
template <typename T>
struct NoInit : std::allocator<T> {
  template <typename U>
  struct rebind { typedef NoInit<U> other; };
  template <typename U, typename... A>
  void construct(U* p, A&&... a) {
    if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
    else ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
template <typename T>
using BookVec = std::vector<T, NoInit<T>>;

template <typename V>
static void reserve_touched(V& v, size_t cap) {
  if (cap <= v.capacity()) return;
  const size_t n = v.size();
  v.reserve(cap);
  v.resize(cap, typename V::value_type());   // first touch of every page, here and not in the replay
  v.resize(n);
}

template <typename V>
static void grow_for(V& v, size_t extra) {   // geometric reserve
  if (v.size() + extra > v.capacity()) reserve_touched(v, std::max(v.size() + extra, 2 * v.capacity()));
}

// Fork-join helpers of the delta replay: T - 1 threads asleep on a condition variable between
// jobs; run(fn) wakes them, runs share 0 itself and returns when every share is done.  One core
// streams a large batch's delta (72 B in, 80 B out per node) at ~13 GB/s; the replay of a 32768-
// record batch took 0.29 ms on it, longer than the GPU step of a rank at 8 ranks.
class ReplayPool {
 public:
  static constexpr int T = 4;
  ~ReplayPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_)
      if (t.joinable()) t.join();
  }
  void run(const std::function<void(int)>& fn) {
    if (th_.empty())
      for (int k = 1; k < T; ++k) th_.emplace_back([this, k] { loop(k); });
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      left_ = T - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int k) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        fn = fn_;
      }
      (*fn)(k);
      {
        std::lock_guard<std::mutex> lk(mu_);
        --left_;
      }
      done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool quit_ = false;
};

struct tr_book {
  std::unique_ptr<ReplayPool> pool;    // started by the first large delta
  BookVec<double> xyt;                 // node poses, insertion order (= G.keys() order)
  BookVec<int64_t> parent;             // cameFrom parent (-1 = None)
  BookVec<double> u6;                  // cameFrom control
  BookVec<int64_t> e_par, e_child;     // edges in append order (G[qnear].append(qnew))
  PoseIndex index;                     // every node
  PoseIndex integral;                  // nodes with integral x and y: the only ones a sample
                                       // ((int x, int y), theta) can equal (rrt.py:151)
  bool straight_reject = false;
  std::vector<uint64_t> hbuf;          // per-record pose hashes (ingest scratch)

  int64_t size() const { return (int64_t)parent.size(); }

  bool same(int64_t i, double x, double y, double t) const {
    const double* p = &xyt[3 * i];
    return dbits(p[0]) == dbits(x) && dbits(p[1]) == dbits(y) && dbits(p[2]) == dbits(t);
  }

  int64_t lookup(const PoseIndex& ix, double x, double y, double t) const {
    return ix.find(key_hash(x, y, t), [&](int64_t i) { return same(i, x, y, t); });
  }

  int64_t add(double x, double y, double t, bool* fresh) { return add_h(key_hash(x, y, t), x, y, t, fresh); }

  int64_t add_h(uint64_t h, double x, double y, double t, bool* fresh) {
    int64_t f = index.find(h, [&](int64_t i) { return same(i, x, y, t); });
    if (f >= 0) {
      *fresh = false;
      return f;
    }
    int64_t i = size();
    xyt.push_back(x);
    xyt.push_back(y);
    xyt.push_back(t);
    parent.push_back(-1);
    u6.resize(u6.size() + 6, 0.0);
    index.insert(h, i);
    if (x == floor(x) && y == floor(y)) integral.insert(h, i);
    *fresh = true;
    return i;
  }

  void reset(const double* s) {
    xyt.clear();
    parent.clear();
    u6.clear();
    e_par.clear();
    e_child.clear();
    index.clear();
    integral.clear();
    bool f;
    add(s[0], s[1], s[2], &f);
  }

  int index_error(int64_t before, int64_t* n_new) {
    *n_new = size() - before;
    return fail(TR_E_INDEX, "index is out of bounds for axis 0 (imarray[y][x], search.py:30)");
  }

  void push_node(double x, double y, double t) {
    xyt.push_back(x);
    xyt.push_back(y);
    xyt.push_back(t);
    parent.push_back(-1);
    u6.resize(u6.size() + 6, 0.0);
  }

  void set_came_from(int64_t i, const tr_record& q) {
    parent[i] = q.near;
    double* u = &u6[6 * i];
    u[0] = q.steer; u[1] = q.iccx; u[2] = q.iccy; u[3] = q.rad; u[4] = q.dist;
    u[5] = (q.flags & TR_FL_STRAIGHT) ? 1.0 : 0.0;
    if (q.flags & TR_FL_STRAIGHT) { u[1] = u[2] = u[3] = 0.0; }
  }

  // Replay of device-resolved records (dedupe.hip): the same decisions as ingest(), in sample
  // order, with the pose lookups already done on the device.  (The pose indexes of this book are
  // not maintained on this path.)
  int replay(const tr_commit_rec* cr, int64_t n, int64_t* n_new, int64_t* sol) {
    const int64_t before = size();
    *sol = -1;
    grow_for(xyt, 3 * (size_t)n);
    grow_for(parent, (size_t)n);
    grow_for(u6, 6 * (size_t)n);
    grow_for(e_par, (size_t)n);
    grow_for(e_child, (size_t)n);
    // Re-reached nodes (duplicates) overwrite cameFrom of an arbitrary earlier node: prefetch
    // those parent/control lines a few records ahead (they miss the cache).
    constexpr int64_t PF = 16;
    auto prefetch = [&](int64_t k) {
      if (k < n && cr[k].r.status == TR_ST_OK && !(cr[k].flags & TR_CI_FIRST)) {
        const int64_t i = cr[k].idx;
        if (i >= 0 && i < size()) {
          __builtin_prefetch(&parent[i], 1);
          __builtin_prefetch(&u6[6 * i], 1);
        }
      }
    };
    for (int64_t k = 0; k < PF; ++k) prefetch(k);
    for (int64_t j = 0; j < n; ++j) {
      prefetch(j + PF);
      const tr_record& q = cr[j].r;
      const int32_t f = cr[j].flags;
      if (cr[j].pad) {
        *n_new = size() - before;
        return fail(TR_E_STATE, dde_message(cr[j].pad));
      }
      if (q.status == TR_ST_SKIP) continue;
      if (q.status == TR_ST_INDEX && (q.flags & TR_FL_INDEX_SAMPLE)) return index_error(before, n_new);
      if (f & TR_CI_MEMBER) continue;                       // "Qrand already in keys"
      if (q.status == TR_ST_INDEX) return index_error(before, n_new);
      if (q.status == TR_ST_STRAIGHT && !straight_reject) {
        *n_new = size() - before;
        return fail(TR_E_STRAIGHT, "unsupported operand type(s) for *: 'float' and 'NoneType'");
      }
      if (q.status != TR_ST_OK) continue;
      const int64_t i = cr[j].idx;
      if (f & TR_CI_FIRST) {
        if (i != size()) {
          *n_new = size() - before;
          return fail(TR_E_STATE, "device node index out of order");
        }
        push_node(q.x, q.y, q.th);
      }
      e_par.push_back(q.near);
      e_child.push_back(i);
      if (!(f & TR_CI_SAME_NEAR)) set_came_from(i, q);
      if (q.flags & TR_FL_GOAL) {
        *sol = i;
        break;
      }
    }
    *n_new = size() - before;
    return TR_OK;
  }

  // Replay of a batch's compact delta (dedupe.hip): its new nodes in index order with their final
  // cameFrom, its edges in sample order, cameFrom overwrites of snapshot nodes in sample order.
  // The same book as replay() of the batch's records (batches without goal / raise only).
  int replay_delta(const DHead& h, const DNode* nd, const DEdge* ed, const DUpd* up, int64_t* n_new) {
    *n_new = 0;
    if (h.n == 0) return TR_OK;          // an empty batch: nothing on the device either
    if (h.base != size())
      return fail(TR_E_STATE, "device node count out of step with the book (device " +
                                  std::to_string(h.base) + ", book " + std::to_string(size()) +
                                  ", batch of " + std::to_string(h.n) + " records, " +
                                  std::to_string(h.n_new) + " new)");
    const size_t nn = (size_t)h.n_new, ne = (size_t)h.n_edge;
    grow_for(xyt, 3 * nn);
    grow_for(parent, nn);
    grow_for(u6, 6 * nn);
    grow_for(e_par, ne);
    grow_for(e_child, ne);
    const size_t b = parent.size();
    xyt.resize(xyt.size() + 3 * nn);
    parent.resize(b + nn);
    u6.resize(u6.size() + 6 * nn);
    double* X = xyt.data() + 3 * b;
    double* U = u6.data() + 6 * b;
    int64_t* Pp = parent.data() + b;
    const size_t eb = e_par.size();
    e_par.resize(eb + ne);
    e_child.resize(eb + ne);
    std::atomic<bool> bad{false};
    // share k of T: a contiguous range of the nodes and of the edges, and the cameFrom overwrites
    // of the nodes idx % T == k (overwrites of one node stay in record order)
    auto share = [&](int k, int T) {
      for (size_t q = nn * k / T; q < nn * (k + 1) / T; ++q) {
        const DNode& d = nd[q];
        X[3 * q] = d.x;
        X[3 * q + 1] = d.y;
        X[3 * q + 2] = d.th;
        Pp[q] = d.parent;
        double* u = U + 6 * q;
        u[0] = d.u[0]; u[1] = d.u[1]; u[2] = d.u[2]; u[3] = d.u[3]; u[4] = d.u[4];
        u[5] = d.straight ? 1.0 : 0.0;
      }
      for (size_t q = ne * k / T; q < ne * (k + 1) / T; ++q) {
        e_par[eb + q] = ed[q].par;
        e_child[eb + q] = ed[q].child;
      }
    };
    auto updates = [&](int k, int T) {
      for (int64_t q = 0; q < h.n_upd; ++q) {
        const DUpd& d = up[q];
        // a snapshot node re-reached, or a new node of this batch reached again (the one-kernel
        // dedupe sends a later record's cameFrom as an update)
        if (d.idx < 0 || d.idx >= (int64_t)(b + nn)) { bad = true; return; }
        if (T > 1 && d.idx % T != k) continue;
        parent[d.idx] = d.parent;
        double* u = &u6[6 * (size_t)d.idx];
        u[0] = d.u[0]; u[1] = d.u[1]; u[2] = d.u[2]; u[3] = d.u[3]; u[4] = d.u[4];
        u[5] = d.straight ? 1.0 : 0.0;
      }
    };
    if (nn + ne >= 16384) {              // large deltas: four cores (the new nodes first: an
      if (!pool) pool.reset(new ReplayPool());       // overwrite may name one of them)
      pool->run([&](int k) { share(k, ReplayPool::T); });
      pool->run([&](int k) { updates(k, ReplayPool::T); });
    } else {
      share(0, 1);
      updates(0, 1);
    }
    if (bad) return fail(TR_E_STATE, "device update out of range");
    *n_new = h.n_new;
    return TR_OK;
  }

  // rrt.py:148-153 (membership), 179-201 (append) for records in sample order.
  int ingest(const tr_sample* s, const tr_record* r, int64_t n, int64_t n_snap, int64_t* n_new,
             int64_t* sol) {
    const int64_t before = size();
    *sol = -1;
    grow_for(xyt, 3 * (size_t)n);
    grow_for(parent, (size_t)n);
    grow_for(u6, 6 * (size_t)n);
    grow_for(e_par, (size_t)n);
    grow_for(e_child, (size_t)n);
    // The appends are a dependent chain of cache-missing probes (pose index, qnear's pose); hash
    // every accepted record first and prefetch PF records ahead.
    constexpr int64_t PF = 24;
    hbuf.resize((size_t)n);
    for (int64_t j = 0; j < n; ++j)
      hbuf[j] = r[j].status == TR_ST_OK ? key_hash(r[j].x, r[j].y, r[j].th) : 0;
    auto prefetch = [&](int64_t k) {
      if (k < n && r[k].status == TR_ST_OK) {
        __builtin_prefetch(&index.slots[hbuf[k] & index.mask]);
        if (r[k].near >= 0 && 3 * r[k].near < (int64_t)xyt.size()) __builtin_prefetch(&xyt[3 * r[k].near]);
      }
    };
    for (int64_t k = 0; k < PF; ++k) prefetch(k);
    for (int64_t j = 0; j < n; ++j) {
      prefetch(j + PF);
      const tr_record& q = r[j];
      if (q.status == TR_ST_SKIP) continue;
      if (q.status == TR_ST_INDEX && (q.flags & TR_FL_INDEX_SAMPLE)) return index_error(before, n_new);
      const int64_t hit = lookup(integral, (double)s[j].x, (double)s[j].y, s[j].th);
      if (hit >= 0 && hit < n_snap) continue;  // "Qrand already in keys"
      if (q.status == TR_ST_INDEX) return index_error(before, n_new);
      if (q.status == TR_ST_STRAIGHT && !straight_reject) {
        *n_new = size() - before;
        return fail(TR_E_STRAIGHT, "unsupported operand type(s) for *: 'float' and 'NoneType'");
      }
      if (q.status != TR_ST_OK) continue;
      bool fresh;
      const int64_t i = add_h(hbuf[j], q.x, q.y, q.th, &fresh);
      e_par.push_back(q.near);
      e_child.push_back(i);
      const double* nr = &xyt[3 * q.near];
      const bool same = dbits(q.x) == dbits(nr[0]) && dbits(q.y) == dbits(nr[1]) &&
                        dbits(q.th) == dbits(nr[2]);
      if (!same) set_came_from(i, q);
      if (q.flags & TR_FL_GOAL) {
        *sol = i;
        break;
      }
    }
    *n_new = size() - before;
    return TR_OK;
  }
};

// ------------------------------------------------------------------ RCCL (multi-GPU exchange)
// The engine owns its communicator for the one exchange of the sharded path (the all-gather of
// every rank's samples and records).  librccl.so.1 is loaded on first use (the one PyTorch already
// mapped, when present: same SONAME), so the library has no link-time dependency on RCCL.
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  const char* (*err)(ncclResult_t) = nullptr;
};

static const Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r.h ? &r : nullptr;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return nullptr;
  r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
  r.init = (decltype(r.init))dlsym(h, "ncclCommInitRank");
  r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
  r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
  r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
  if (!r.get_id || !r.init || !r.all_gather || !r.destroy || !r.err) return nullptr;
  r.h = h;
  return &r;
}

// ------------------------------------------------------------------ static scratch
// tr_expand_dev_noalloc's scratch: one file-scope device array per GPU (every GPU the library's
// code object is loaded on holds its own copy, at its own address, until the process ends).  In
// host code the array's name is only a handle for hipGetSymbolAddress: tr_create resolves it once
// per device, with that device current, and everything else uses the resolved pointer.
constexpr size_t NOALLOC_BYTES = 16u << 20;
static __device__ __align__(256) unsigned char scratch[NOALLOC_BYTES];
constexpr int NOALLOC_MAX_DEV = 64;
static unsigned char* g_scratch_ptr[NOALLOC_MAX_DEV] = {};
static std::mutex g_scratch_mu;

static int scratch_resolve(int device) {       // the caller has made `device` current
  if (device < 0 || device >= NOALLOC_MAX_DEV) return TR_OK;   // no scratch there: noalloc refuses
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  if (g_scratch_ptr[device]) return TR_OK;
  void* p = nullptr;
  HIPCHK(hipGetSymbolAddress(&p, HIP_SYMBOL(scratch)));
  g_scratch_ptr[device] = static_cast<unsigned char*>(p);
  return TR_OK;
}

// ------------------------------------------------------------------ context
struct tr_ctx {
  int device = 0;
  hipStream_t own = nullptr, st = nullptr;
  Params P{};
  bool have_grid = false;
  int64_t H = 0, W = 0;
  DBuf<uint32_t> grid;                 // bit-packed occupancy (geom.hpp Grid)
  std::vector<uint32_t> hbits;         // the same words on the host (tr_lineofsight, tr_astar)
  std::vector<uint8_t> hgrid;          // the caller's bytes: the Theta* search's neighbour tests
  // device tree (insertion order = rrt.py G.keys() order) and its pose table
  DBuf<double2> txy;   // node (x, y) fp64
  DBuf<float4> t4;     // the NN screen's operand (screen_node: centred fp32 x, y, |.|^2)
  int32_t cx = 0, cy = 0;   // tree centre of the screen, fixed from one tree reset to the next
  DBuf<double> tth;
  int64_t N = 0;       // nodes committed on the host (== device count outside a pipelined session)
  int64_t n_ub = 0;    // upper bound of the device count (batches in flight included)
  DBuf<int64_t> d_count;
  DBuf<unsigned long long> d_maxabs;
  DBuf<PoseSlot> htab;
  DBuf<unsigned long long> btab, blast;   // batch tables of large batches (dedupe.hip)
  uint64_t hmask = 0, bmask = 0;
  unsigned long long epoch = 0;
  DBuf<int32_t> dd_slot, dd_lr, dd_bc;  // large-batch scratch: table slot, local ranks, block counts
  DBuf<int32_t> dd_err;                // device bookkeeping error bits (TR_DDE_*), sticky
  DBuf<int64_t> dd_base;
  DBuf<unsigned long long> dd_special;
  // Per-context options (tr_set_option).  gate: the cross-stream edges of the pipelined loop go
  // through stream gates (k_gate / flags) instead of events; switched off by tr_create when the
  // device serializes dispatches across streams (gate_probe: counter-collecting profilers do).
  bool gate = true;
  bool fused_delta = true;             // look-ahead correction inside k_expand_arc (else k_nn_delta)
  // The appended nodes by bin (thetarrt_internal.hpp: DeltaBins), built by k_dd and read by the
  // fused correction.  db_ok[s] = the dedupe epoch whose nodes set s holds (0: none), db_zero[s] =
  // the epoch set s's counts were zeroed for.
#ifdef TR_DIAG_NOBINS                        // diagnosis builds only: the option starts at 0
  bool delta_bins = false;
#else
  bool delta_bins = true;              // tr_set_option "delta_bins"
#endif
  DBuf<uint32_t> db_cnt;
  DBuf<DBItem> db_items, db_ovf;
  int32_t db_ovf_cap = 0;
  int32_t db_shift = 0, db_nbx = 0, db_nby = 0;
  int64_t db_for_n = 0;                // records per batch the bin size was chosen for
  unsigned long long db_ok[4] = {}, db_zero[4] = {};
  DeltaBins bins_view() const {
    DeltaBins b;
    b.cnt = db_cnt.p;
    b.items = db_items.p;
    b.ovf = db_ovf.p;
    b.ovf_cap = db_ovf_cap;
    b.shift = db_shift;
    b.nbx = db_nbx;
    b.nby = db_nby;
    b.xmax = (int32_t)H - 1;
    b.ymax = (int32_t)W - 1;
    return b;
  }
  // Nearest nodes from cell lists over the map (nn_grid.hip) instead of the sweep of every node:
  // brought up to date from the tree before every query batch, set 0 on the context stream, set 1
  // on the look-ahead stream (each stream's builds and queries follow one another).  A build
  // merges the nodes appended since the set's last build into item / start buffers [par ^ 1] and
  // leaves its node count in built[par ^ 1]; `full` builds take every node (after a tree reset:
  // tree_gen, a map or cell-size change, a reallocation).
  bool nn_grid = true;                 // tr_set_option "nn_grid"
  // Samples whose second pass is long (far from every node, or next to a cell where the tree piles
  // up) are scanned by their block (small batches: nothing more to launch on the look-ahead stream)
  // or, from this global batch size on (tr_set_option "nn_far_sweep"), collected in a list that the
  // sweep's two kernels take: a sample far from every node reads a ring of cells that grows with
  // the square of its distance, and a tree that has saturated its map leaves thousands of such
  // samples per batch, which the matrix screen handles at a fixed cost per pair.
  int64_t nn_far_sweep = 8193;
  // ... the samples whose second pass covers more nodes than this ("nn_far_nodes"; shorter passes
  // stay with the block: the sweep's resolve rescans whole chunks per candidate, so it only pays
  // for the long ones.  Measured, M expansions/s at thresholds 4096 / 12288 / 65536: 32768 samples
  // 56.3 / 55.5 / 42.5, 16384 samples 59.9 / 60.6 / 61.8, 65536 samples 35.5 / 39.3 / 22.8, cfg3
  // 21.8 / 24.6 / 19.3; every sample through the sweep: 41.0 / 39.9 / 30.2 / 15.3)
  int64_t nn_far_nodes = 12288;
  int64_t nn_grid_min = -1;            // nodes from which they are used (< 0: a node per 8 pixels)
  unsigned long long tree_gen = 1;     // bumped by every tree reset
  struct CellSet {
    DBuf<uint32_t> cnt, shift, rank, start[2];
    DBuf<DBItem> items[2];
    DBuf<int64_t> built;               // [2]
    DBuf<unsigned long long> part;     // the scan's block sums
    DBuf<int32_t> far_n, far_j;        // the far list of a query batch: count, sample indices
    DBuf<int2> far_q;                  // ... and their pixels
    uint32_t serial = 0;               // builds so far
    NNGrid g;                          // plan (cs, P, xmax, ymax) of the last build
    bool moved = true;                 // buffers (re)allocated since the last build
    int par = 0;                       // buffers holding the last build
    unsigned long long gen = 0;        // tree_gen of the last build (0: none)
    int64_t for_n = 0;                 // node bound the cell size was chosen for
  } cells[2];
  bool dd_fused = true;                // one-kernel dedupe k_dd (else claim / count / emit)
  bool dd_gatefold = true;             // the next batch's gate rides at the end of k_dd
  int64_t dd_fused_max = 8192;         // records per batch up to which k_dd is used
  bool replay_on = true;               // the host book follows the device tree (tr_set_option "book")
  unsigned long long gated_seq = 0;    // the look-ahead seq the last k_dd waited for
  DBuf<int32_t> dd_ticket;
  DBuf<unsigned long long> dd_bst;
  DBuf<int64_t> dd_idx;
  DBuf<unsigned long long> st_done;    // gate flag: seq of the latest look-ahead finished
  DBuf<int32_t> st_blocks;             // resolve blocks finished (the last one publishes st_done)
  unsigned long long st_seq = 0;
  DBuf<unsigned long long> dd_done;
  DBuf<int32_t> dd_blocks;
  // batch scratch
  DBuf<int2> qxy;
  DBuf<int32_t> live, err;
  DBuf<float> m32;
  DBuf<int64_t> iout, cnt;
  DBuf<tr_sample> samp;
  DBuf<tr_record> rec, rec_all;
  DBuf<double> gauss, fin, fout;
  DBuf<uint8_t> bout;
  DBuf<int32_t> i32;
  HBuf<double> h_x;
  // findnearest (rrt.py:117-128): edges (parent, child), poses, goals, partials, results
  DBuf<int64_t> fn_par, fn_child, fn_out;
  DBuf<double> fn_pose, fn_goal, fn_d;
  DBuf<uint8_t> fn_part;
  // tr_astar_batch: per-query queue / gScore / state memory and the staged queries and results
  DBuf<uint8_t> as_work;
  DBuf<int32_t> as_sg;
  DBuf<int64_t> as_path, as_len, as_stats;
  // session: host book + a ring of pinned commit slots (records + device resolution)
  static constexpr int R = 6;
  // commit slot k: DHead, then per record capacity DNode, DEdge, DUpd, tr_resolved (special
  // batches only) arrays, in pinned host memory written by the device (zero-copy)
  HBuf<uint8_t> r_cr[R];
  int64_t r_cap[R] = {};
  hipEvent_t r_ev[R] = {};
  int64_t r_n[R] = {};
  // gate mode: the device stores the batch's epoch into r_ready[k] (pinned) when commit slot k is
  // complete; the worker polls it instead of synchronizing on an event (no marker on the stream)
  HBuf<unsigned long long> r_ready;
  std::atomic<long long> head_waits{0};   // batches whose head arrived after their ready flag
  unsigned long long r_epoch[R] = {};
  hipStream_t r_stream[R] = {};
  int r_head = 0, r_tail = 0, r_count = 0;
  // Replay worker: a host thread replays each deduplicated batch into the book as soon as its
  // records land (in ring order), so the thread that enqueues batches never runs the replay.
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  bool quit = false;
  int w_next = 0, w_pending = 0;       // next ring slot to replay, slots queued
  bool r_done[R] = {};
  int r_rc[R] = {};
  int64_t r_nnew[R] = {}, r_sol[R] = {}, r_nodes[R] = {}, r_devnew[R] = {};
  double r_rep_us[R] = {};
  std::string r_msg[R];
  int64_t w_dev_nodes = 1;             // worker: device node count after the last replayed batch
  int book_err = 0;                    // first replay error (the session stops there)
  std::string book_msg;
  int64_t book_sol = -1;               // goal node of the first batch that reached it
  tr_book book;
  bool session = false;
  double goal[3] = {0, 0, 0};
  int timing = 0;                      // 1: time the NN; 2: every phase (events cost GPU gaps)
  uint32_t tmask = 3;                  // level 1 samples batches with (seq & tmask) == 0
  hipEvent_t t_ev[6] = {};
  double t_us[5] = {0, 0, 0, 0, 0};    // last batch: nn, expand, arc, dedupe, total (us)
  double host_us[3] = {0, 0, 0};       // last commit: wait, replay, other
  // staged NN sweeps: a low-priority side stream screens future batches (up to SQ ahead) against
  // the tree after the latest enqueued dedupe while the current batch expands; the expand of a
  // staged batch then sweeps only the nodes appended since its snapshot (the delta)
  static constexpr int SQ = 2, NS = SQ + 1;   // look-ahead depth, per-batch scratch sets
  hipStream_t side = nullptr;
  hipEvent_t ev_dd = nullptr;
  hipEvent_t ev_latest = nullptr;      // recorded after the latest dedupe (or the session start)
  DBuf<int64_t> snap;                  // node count after each dedupe, slot epoch % 4
  DBuf<int2> s_qxy[NS];
  DBuf<int32_t> s_live[NS];
  DBuf<float> s_m32[NS];
  DBuf<int64_t> s_near[NS];            // nearest node per sample (look-ahead, then corrected)
  DBuf<double> s_dnear[NS];            // its exact squared distance
  DBuf<int32_t> chg, n_chg;            // samples whose nearest node changed after the look-ahead
  int next_k = 0;                      // scratch set of the next batch (round robin)
  struct Stage {
    const double* gauss = nullptr;
    int64_t B = 0;
    tr_sample* smp = nullptr;
    tr_record* rec = nullptr;
    int k = 0, slot = 0;
    NNPlan plan;
    int64_t n_lb = 0;                  // lower bound of the snapshot (committed nodes)
    unsigned long long epoch = 0;      // dedupe epoch at stage time (its snapshot slot: epoch & 3)
    unsigned long long seq = 0;        // gate mode: st_done value published after its kernels
    hipEvent_t ev = nullptr;           // event mode: recorded after its kernels on the side stream
  } stq[SQ];                           // staged batches, oldest first
  int st_n = 0;
  int alloc_k() {
    const int k = next_k;
    next_k = (next_k + 1) % NS;
    return k;
  }
  // every staged sweep of a tr_rrt_run timed: a ring of (before pass1, after pass1, after resolve)
  // event triples, harvested when a slot is reused and at the end of the run
  static constexpr int TS = 8;
  hipEvent_t ts_ev[TS][3] = {};
  bool ts_used[TS] = {};
  int ts_next = 0;
  double ts_sum[2] = {0, 0};           // pass1, resolve (us)
  int64_t ts_n = 0;
  int ts_last = -1;                    // slot of the latest timed look-ahead
  int64_t stage_seq = 0;
  // main-stream kernels of every 4th staged batch timed the same way (timing level 1): events
  // [0] before k_nn_delta, [1] before k_expand_arc, [2] after it, [3] before the dedupe, [4] after
  static constexpr int TM = 8;
  hipEvent_t tm_ev[TM][5] = {};
  bool tm_used[TM] = {};
  int tm_next = 0, tm_pending = -1;
  double tm_sum[3] = {0, 0, 0};        // k_nn_delta, k_expand_arc, dedupe (us)
  int64_t tm_n = 0, main_seq = 0;
  bool last_staged = false;            // the last expand used a look-ahead
  ncclComm_t comm = nullptr;            // tr_comm_init: sample-sharded multi-GPU session
  tr_host_gather_fn hg_fn = nullptr;   // tr_comm_init_host: the same exchange through the host
  void* hg_user = nullptr;
  HBuf<uint8_t> hg_send, hg_recv;
  int rank = 0, world = 1;
  bool sharded() const { return comm != nullptr || hg_fn != nullptr; }
  double run_us[5] = {}, run_nn[3] = {}, run_host[3] = {};   // tr_rrt_run statistics
  int64_t run_n = 0;
  // TR_TRACE=1: host timestamps of the last tr_rrt_run's batches, printed to stderr at its end
  // (diagnosis only): [0] enqueue start, [1] expand enqueued, [2] stage enqueued, [3] dedupe
  // enqueued, [4] commit returned; worker: [5] batch event ready, [6] replay done.
  static constexpr int TRN = 256;
  double trc[TRN][7] = {};
  bool trace_on = false;               // tr_set_option "trace"
  int stage_n = 0;                     // ... look-aheads of the current run so far
  double trace_t0 = 0;                 // ... the run's entry
  int64_t rep_seq = 0, enq_seq = 0, com_seq = 0;   // trace rows: replayed, enqueued, committed
  double nn_us[3] = {0, 0, 0};         // last batch: staged sweep (side), NN on the batch's path
  double stage_us[5] = {};             // TR_TRACE: stage_batch's calls (wait, samples, sweep, resolve, record)
  // Device gaussian stream (rng.hip): numpy's RandomState state -> rand_conf's draws on the GPU.
  // tr_rrt_run without caller gaussians draws each chunk of RC batches on its own stream, one
  // chunk ahead, into two chunk slots; rng_pos[0] = the stream position between calls,
  // rng_pos[1 + (q & 7) RC + b] = position after batch b of chunk q and rng_keys its key block
  // (kept 8 chunks: a run rewinds to the batch that reached the goal, up to `lag` batches back,
  // by re-seeding the ring there), [1 + 8 RC] scratch.
  static constexpr int RC = 8;
  // gate mode: a run's first batch of gaussians is handed to the context stream through a polled
  // flag (k_publish on the rng stream, k_gate on the context stream) instead of an event: the
  // event's edge costs ~25 us at the one point of a run where nothing else is in flight
  DBuf<unsigned long long> rng_flag;
  unsigned long long rng_seq = 0;
  hipStream_t rng_st = nullptr;
  bool rng_on = false;
  DBuf<uint32_t> rng_ring;             // raw MT19937 words, word w at [w mod rng_rs]
  int64_t rng_rs = 0;
  DBuf<int64_t> rng_gen;               // words generated (the ring's end, a multiple of 624)
  DBuf<RngPos> rng_pos;
  DBuf<int32_t> rng_cnt, rng_err, rng_done;
  DBuf<uint32_t> rng_seeds;            // the generator workgroups' jumped state blocks (rng.hip)
  DBuf<uint32_t> rng_keys;             // key block of every rng_pos[1 + i] batch end (624 words)
  DBuf<double> rng_out;                // 2 chunk slots of RC x 3 BT gaussians
  hipEvent_t rng_ev[2] = {}, rng_free = nullptr;
  hipEvent_t rng_b[RC] = {};           // a run's first chunk is drawn batch by batch: one event each
  HBuf<int32_t> rng_err_h;             // the stream's error word, copied at the end of a run

  Grid G() const { return Grid{grid.p, H, W, (W + 31) / 32}; }
  Grid HG() const { return Grid{hbits.data(), H, W, (W + 31) / 32}; }
  CommitOut commit_view(int k) const {
    uint8_t* p = r_cr[k].p;
    const int64_t cap = r_cap[k];
    CommitOut o;
    o.head = reinterpret_cast<DHead*>(p);
    o.nodes = reinterpret_cast<DNode*>(p + 64);
    o.edges = reinterpret_cast<DEdge*>(p + 64 + sizeof(DNode) * cap);
    o.upd = reinterpret_cast<DUpd*>(p + 64 + (sizeof(DNode) + sizeof(DEdge)) * cap);
    o.res = reinterpret_cast<tr_resolved*>(p + 64 + (sizeof(DNode) + sizeof(DEdge) + sizeof(DUpd)) * cap);
    return o;
  }
};

static double now_us();

// A special batch's resolved records in order, without a book: what stops the loop there, decided
// as tr_book::replay decides it (the goal's node index, or the error the reference raises).
static int scan_special(const tr_commit_rec* cr, int64_t n, bool straight_reject, int64_t* sol) {
  *sol = -1;
  for (int64_t j = 0; j < n; ++j) {
    const tr_record& q = cr[j].r;
    if (cr[j].pad) return fail(TR_E_STATE, dde_message(cr[j].pad));
    if (q.status == TR_ST_SKIP) continue;
    const bool index_sample = q.status == TR_ST_INDEX && (q.flags & TR_FL_INDEX_SAMPLE);
    if (index_sample || (q.status == TR_ST_INDEX && !(cr[j].flags & TR_CI_MEMBER)))
      return fail(TR_E_INDEX, "index is out of bounds for axis 0 (imarray[y][x], search.py:30)");
    if (cr[j].flags & TR_CI_MEMBER) continue;
    if (q.status == TR_ST_STRAIGHT && !straight_reject)
      return fail(TR_E_STRAIGHT, "unsupported operand type(s) for *: 'float' and 'NoneType'");
    if (q.status == TR_ST_OK && (q.flags & TR_FL_GOAL)) {
      *sol = cr[j].idx;
      break;
    }
  }
  return TR_OK;
}

// Gate mode: spin (then yield) until the device has published batch k's commit slot; after ~2 s
// synchronize the batch's stream (a faulted or hung batch returns an error there) and look again.
static bool wait_ready(tr_ctx* c, int k) {
  const unsigned long long want = c->r_epoch[k];
  auto ready = [&] { return __atomic_load_n(c->r_ready.p + k, __ATOMIC_ACQUIRE) >= want; };
  const double t0 = now_us();
  for (int64_t n = 0; !ready(); ++n) {
    if (n < 4096) {
      __builtin_ia32_pause();
    } else {
      std::this_thread::yield();
      if (now_us() - t0 > 2e6) {
        if (hipStreamSynchronize(c->r_stream[k]) != hipSuccess) return false;
        return ready();
      }
    }
  }
  return true;
}

// The slot's head must be the one this batch's dedupe wrote.  The ready flag (or the event) orders
// it after the head on the device; should the host still see the head of the slot's earlier use,
// the worker waits for the right one (2 s at most) instead of replaying a stale delta, and counts
// the occurrence (tr_get_option "head_waits").
static bool wait_head(tr_ctx* c, int k) {
  const int32_t want = head_tag(c->r_epoch[k]);
  const int32_t* tag = &c->commit_view(k).head->pad;
  if (__atomic_load_n(tag, __ATOMIC_ACQUIRE) == want) return true;
  c->head_waits.fetch_add(1, std::memory_order_relaxed);
  const double t0 = now_us();
  while (__atomic_load_n(tag, __ATOMIC_ACQUIRE) != want) {
    if (now_us() - t0 > 2e6) return false;
    __builtin_ia32_pause();
  }
  // (the slot's other stores left the device before the head's: a moment for them as well)
  for (const double t1 = now_us(); now_us() - t1 < 5.0;) __builtin_ia32_pause();
  return true;
}

static void replay_worker(tr_ctx* c) {
  (void)hipSetDevice(c->device);
  for (;;) {
    int k;
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv_work.wait(lk, [c] { return c->quit || c->w_pending > 0; });
      if (c->w_pending == 0) return;         // quit with nothing left
      k = c->w_next;
    }
    if (c->gate) {
      if (!wait_ready(c, k)) {
        std::lock_guard<std::mutex> lk(c->mu);   // the batch never completed: fail it
        c->r_done[k] = true;
        c->r_rc[k] = TR_E_HIP;
        c->r_msg[k] = "device pipeline: a batch did not complete (" +
                      std::string(hipGetErrorString(hipGetLastError())) + ")";
        c->r_devnew[k] = c->r_nnew[k] = 0;
        c->r_sol[k] = -1;
        c->r_nodes[k] = c->book.size();
        c->r_rep_us[k] = 0;
        c->w_next = (k + 1) % tr_ctx::R;
        c->w_pending--;
        c->cv_done.notify_all();
        continue;
      }
    } else {
      (void)hipEventSynchronize(c->r_ev[k]);
    }
    const bool head_ok = wait_head(c, k);
    const double t0 = now_us();
    if (c->trace_on) c->trc[c->rep_seq % tr_ctx::TRN][5] = t0;
    int rc = TR_OK;
    int64_t n_new = 0, sol = -1;
    std::string msg;
    if (!head_ok && !c->book_err) {          // nothing of this slot can be trusted
      c->book_err = TR_E_HIP;
      c->book_msg = "device pipeline: a batch's commit slot never showed its head";
    }
    if (c->book_err) {                       // the reference raised in an earlier batch
      rc = c->book_err;
      msg = c->book_msg;
    } else if (c->book_sol >= 0) {           // goal found earlier: later batches are not appended
      sol = c->book_sol;
    } else if (!c->replay_on) {
      // this context keeps no host book (tr_set_option "book" 0: the ranks of a sharded run other
      // than the one that reports the tree): only what stops the loop is read, in record order
      const CommitOut v = c->commit_view(k);
      if (v.head->err) {
        rc = fail(TR_E_STATE, dde_message(v.head->err));
      } else if (v.head->special) {
        rc = scan_special(v.res, c->r_n[k], c->book.straight_reject, &sol);
      }
      if (rc) { msg = g_err; c->book_err = rc; c->book_msg = msg; }
      if (sol >= 0) c->book_sol = sol;
    } else {
      try {
        const CommitOut v = c->commit_view(k);
        if (v.head->err) {
          rc = fail(TR_E_STATE, dde_message(v.head->err));
        } else if (v.head->special) {  // goal / raise / error in the batch: every record in order
          rc = c->book.replay(v.res, c->r_n[k], &n_new, &sol);
        } else {
          rc = c->book.replay_delta(*v.head, v.nodes, v.edges, v.upd, &n_new);
        }
        if (rc) msg = g_err;
      } catch (const std::exception& ex) {
        rc = TR_E_HIP;
        msg = ex.what();
      }
      if (rc) { c->book_err = rc; c->book_msg = msg; }
      if (sol >= 0) c->book_sol = sol;
    }
    // nodes the device appended for this batch (all first occurrences, also past a goal or an
    // error where the book stops): keeps n_ub an upper bound of the device count
    int64_t dev_new = 0;
    dev_new = c->commit_view(k).head->n_new;
    const double t1 = now_us();
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->r_done[k] = true;
      c->r_devnew[k] = dev_new;
      c->r_rc[k] = rc;
      c->r_msg[k] = msg;
      c->r_nnew[k] = n_new;
      c->r_sol[k] = sol;
      const DHead* hd = c->commit_view(k).head;
      if (hd->n) c->w_dev_nodes = hd->base + hd->n_new;   // (an empty batch leaves the count)
      c->r_nodes[k] = c->replay_on ? c->book.size() : c->w_dev_nodes;
      c->r_rep_us[k] = t1 - t0;
      if (c->trace_on) c->trc[c->rep_seq++ % tr_ctx::TRN][6] = t1;
      c->w_next = (k + 1) % tr_ctx::R;
      c->w_pending--;
    }
    c->cv_done.notify_all();
  }
}

static void worker_start(tr_ctx* c) {
  if (!c->worker.joinable()) c->worker = std::thread(replay_worker, c);
}

static void worker_drain(tr_ctx* c) {        // every queued batch replayed
  std::unique_lock<std::mutex> lk(c->mu);
  c->cv_done.wait(lk, [c] { return c->w_pending == 0; });
}

static void worker_stop(tr_ctx* c) {
  if (!c->worker.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->quit = true;
  }
  c->cv_work.notify_all();
  c->worker.join();
}

static int set_dev(tr_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return TR_OK;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename T>
static hipError_t regrow(hipStream_t st, DBuf<T>& b, int64_t keep, int64_t cap) {
  T* q = nullptr;
  hipError_t e = hipMalloc(&q, sizeof(T) * (size_t)cap);
  if (e != hipSuccess) return e;
  if (keep) {
    e = copy_sync(st, q, b.p, sizeof(T) * (size_t)keep, hipMemcpyDeviceToDevice);
    if (e != hipSuccess) return e;
  }
  if (b.p) (void)hipFree(b.p);
  b.p = q;
  b.cap = cap;
  return hipSuccess;
}

static uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1024;
  while (p < v) p <<= 1;
  return p;
}

// Device tree arrays hold >= need nodes (stalls the stream when it has to grow).
static int ensure_tree(tr_ctx* c, int64_t need) {
  if (need <= c->txy.cap && need <= c->t4.cap && need <= c->tth.cap) return TR_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->side));     // a staged sweep reads the tree
  const int64_t cap = std::max<int64_t>(need, 2 * c->txy.cap);
  const int64_t keep = std::min(c->n_ub, c->txy.cap);
  HIPCHK(regrow(c->st, c->txy, keep, cap));
  HIPCHK(regrow(c->st, c->t4, keep, cap));
  HIPCHK(regrow(c->st, c->tth, keep, cap));
  return TR_OK;
}

// Pose table load <= 1/2 for `need` nodes; a grown table is rebuilt from the device tree.
static int ensure_table(tr_ctx* c, int64_t need) {
  if (c->htab.p && (uint64_t)(2 * need) <= c->hmask + 1) return TR_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  const uint64_t slots = pow2_at_least((uint64_t)(4 * std::max<int64_t>(need, 1)));
  c->htab.release();
  HIPCHK(c->htab.reserve((int64_t)slots));
  c->hmask = slots - 1;
  int64_t n = 0;
  HIPCHK(copy_sync(c->st, &n, c->d_count.p, sizeof(int64_t), hipMemcpyDeviceToHost));
  dd_rebuild(c->st, c->htab.p, c->hmask, c->dd_err.p, c->txy.p, c->tth.p, n);
  HIPCHK(hipGetLastError());
  return TR_OK;
}

static int ensure_dd_scratch(tr_ctx* c, int64_t n) {
  HIPCHK(c->dd_base.reserve(1));
  if (!c->dd_special.p) {
    HIPCHK(c->dd_special.reserve(1));
    HIPCHK(fill_sync(c->st, c->dd_special.p, 0, sizeof(unsigned long long)));
    HIPCHK(c->dd_blocks.reserve(1));
    HIPCHK(fill_sync(c->st, c->dd_blocks.p, 0, sizeof(int32_t)));
  }
  if (!c->dd_ticket.p) {
    HIPCHK(c->dd_ticket.reserve(1));
    HIPCHK(fill_sync(c->st, c->dd_ticket.p, 0, sizeof(int32_t)));
  }
  const int64_t m = std::max<int64_t>(n, 1);
  if (m > c->dd_slot.cap) {                      // in use by batches in flight: wait for them
    HIPCHK(hipStreamSynchronize(c->st));
    HIPCHK(c->dd_slot.reserve(m));
    HIPCHK(c->dd_lr.reserve(3 * m));
    HIPCHK(c->dd_idx.reserve(m));
    const int64_t nb = (m + DD_BLOCK - 1) / DD_BLOCK;   // status words: epoch-tagged, zeroed once
    HIPCHK(c->dd_bc.reserve(3 * nb));
    if (nb > c->dd_bst.cap) {
      c->dd_bst.release();
      HIPCHK(c->dd_bst.reserve(nb));
      HIPCHK(fill_sync(c->st, c->dd_bst.p, 0, sizeof(unsigned long long) * c->dd_bst.cap));
    }
  }
  const uint64_t slots = pow2_at_least((uint64_t)(2 * std::max<int64_t>(n, 1)));
  if ((uint64_t)c->btab.cap < slots) {       // epoch-tagged: zeroed once, never cleared per batch
    HIPCHK(hipStreamSynchronize(c->st));
    c->btab.release();
    c->blast.release();
    HIPCHK(c->btab.reserve((int64_t)slots));
    HIPCHK(c->blast.reserve((int64_t)slots));
    HIPCHK(fill_sync(c->st, c->btab.p, 0, sizeof(unsigned long long) * slots));
    HIPCHK(fill_sync(c->st, c->blast.p, 0, sizeof(unsigned long long) * slots));
  }
  c->bmask = (uint64_t)c->btab.cap - 1;      // cap is a power of two (reserve(slots) exact)
  return TR_OK;
}

// Bins for the nodes a dedupe of n records appends: two to three nodes per bin at a 0.6 acceptance
// (side 2^shift pixels, 4 to 256; the corner and border bins of clipped samples take far more, up
// to DB_CAP items, the rest in the set's overflow list, which holds a whole batch).  Re-planned when the batch size moves by more than 4x; a fresh
// allocation holds no epoch (db_ok = 0: the correction scans the nodes until k_dd has filled it).
static int ensure_bins(tr_ctx* c, int64_t n) {
  if (!c->delta_bins || !c->have_grid || n <= 0 || c->H > (1 << 20) || c->W > (1 << 20)) return TR_OK;
  if (c->db_cnt.p && n <= 4 * c->db_for_n && c->db_for_n <= 4 * n && n <= c->db_ovf_cap &&
      c->db_nbx == (int32_t)(((c->H - 1) >> c->db_shift) + 1) &&
      c->db_nby == (int32_t)(((c->W - 1) >> c->db_shift) + 1))
    return TR_OK;
  const double side = std::sqrt(4.0 * (double)c->H * (double)c->W / (0.6 * (double)n));
  int32_t shift = 2;
  while (shift < 8 && (double)(2 << shift) <= side) ++shift;
  HIPCHK(hipStreamSynchronize(c->st));
  c->db_shift = shift;
  c->db_nbx = (int32_t)(((c->H - 1) >> shift) + 1);
  c->db_nby = (int32_t)(((c->W - 1) >> shift) + 1);
  c->db_for_n = n;
  const int64_t nb = (int64_t)c->db_nbx * c->db_nby;
  c->db_cnt.release();
  c->db_items.release();
  c->db_ovf.release();
  c->db_ovf_cap = (int32_t)std::min<int64_t>(4 * n, INT32_MAX);   // >= the nodes a batch appends
  HIPCHK(c->db_cnt.reserve(4 * (nb + 1)));
  HIPCHK(c->db_items.reserve(4 * nb * DB_CAP));
  HIPCHK(c->db_ovf.reserve(4 * (int64_t)c->db_ovf_cap));
  for (int q = 0; q < 4; ++q) c->db_ok[q] = c->db_zero[q] = 0;
  return TR_OK;
}

static int ensure_slot(tr_ctx* c, int k, int64_t n) {
  if (n <= c->r_cap[k] && c->r_cr[k].p) return TR_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  const int64_t cap = std::max<int64_t>(n, 1);
  const int64_t bytes = 64 + cap * (int64_t)(sizeof(DNode) + sizeof(DEdge) + sizeof(DUpd) +
                                             sizeof(tr_resolved));
  c->r_cr[k].release();
  HIPCHK(c->r_cr[k].reserve(bytes));
  c->r_cap[k] = cap;
  return TR_OK;
}

static int need_grid(tr_ctx* c) {
  if (!c) return fail(TR_E_ARG, "ctx is NULL");
  if (!c->have_grid) return fail(TR_E_STATE, "no grid: call tr_set_grid first");
  return set_dev(c);
}

static int check_err_word(tr_ctx* c) {
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, c->err.p, 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  if (e) return fail(TR_E_INDEX, "index is out of bounds (imarray[y][x], search.py:30)");
  return TR_OK;
}

// Grow a session buffer; waits for both streams first (an old buffer may still be in use).
template <typename T>
static int grow(tr_ctx* c, DBuf<T>& b, int64_t n) {
  if (n <= b.cap) return TR_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->side));
  HIPCHK(b.reserve(n));
  return TR_OK;
}

// The nearest-node queries of this context go through cell lists (else through the sweep): a map
// is set (the cells tile it), its sides bound the cell arrays (a map of up to 8192 pixels a side:
// the padded square of cells holds at most 64M, and that only for a tree of a node per pixel), and
// node indices fit 32 bits.
static bool cells_possible(const tr_ctx* c) {
  return c->nn_grid && c->have_grid && c->H <= 8192 && c->W <= 8192 &&
         c->n_ub < (int64_t)INT32_MAX && c->txy.cap < (int64_t)INT32_MAX;
}
// ... and the tree is dense enough on its map (option "nn_grid_min", by default a node per 8
// pixels): while it is sparse, most samples are far from every node, each query takes several
// dependent passes (100 us per batch at 12k nodes on 512 x 512 against 25 us at 60k), and a sweep
// of so few nodes is cheap.
static int64_t cells_min_nodes(const tr_ctx* c) {
  return c->nn_grid_min >= 0 ? c->nn_grid_min : c->H * c->W / 8;
}
enum NNMode { NN_SWEEP, NN_CELLS, NN_CELLS_FAR_SWEEP };
static NNMode nn_mode(const tr_ctx* c, int64_t B) {
  if (!cells_possible(c) || c->n_ub < cells_min_nodes(c)) return NN_SWEEP;
  return B * std::max(c->world, 1) >= c->nn_far_sweep ? NN_CELLS_FAR_SWEEP : NN_CELLS;
}

// Cell set s brought up to date with the nodes [0, *hi_p) on stream st (launches only) -> g for
// the queries.  The cell side is re-planned when the node bound has doubled (or fallen 8x) or the
// map changed; the buffers hold the finest cells the reserved tree can ask for, so a tree that
// fills its reservation never reallocates.
static int cells_alloc(tr_ctx* c, int s) {
  tr_ctx::CellSet& cs = c->cells[s];
  NNGrid top;
  nn_grid_plan(top, c->H, c->W, 2 * std::max(std::max<int64_t>(c->n_ub, 1), c->txy.cap));
  const int64_t words = (int64_t)top.P * top.P + 1;
  const void* before[5] = {cs.cnt.p, cs.start[0].p, cs.items[0].p, cs.built.p, cs.part.p};
  if (int e = grow(c, cs.cnt, words)) return e;
  if (int e = grow(c, cs.shift, words)) return e;
  if (int e = grow(c, cs.rank, c->txy.cap)) return e;
  if (int e = grow(c, cs.built, 2)) return e;
  if (int e = grow(c, cs.part, nn_grid_scan_blocks(top))) return e;
  for (int q = 0; q < 2; ++q) {
    if (int e = grow(c, cs.start[q], words)) return e;
    if (int e = grow(c, cs.items[q], c->txy.cap)) return e;
  }
  if (before[0] != cs.cnt.p || before[1] != cs.start[0].p || before[2] != cs.items[0].p ||
      before[3] != cs.built.p || before[4] != cs.part.p)
    cs.moved = true;                             // the next build starts over (and zeroes the counts)
  return TR_OK;
}

static int cells_build(tr_ctx* c, int s, hipStream_t st, const int64_t* hi_p, NNGrid& g,
                       int64_t far_cap = 0) {
  tr_ctx::CellSet& cs = c->cells[s];
  const int64_t n = std::max<int64_t>(c->n_ub, 1);
  if (int e = cells_alloc(c, s)) return e;
  if (far_cap > 0) {
    if (int e = grow(c, cs.far_n, 1)) return e;
    if (int e = grow(c, cs.far_j, far_cap)) return e;
    if (int e = grow(c, cs.far_q, far_cap)) return e;
  }
  const bool moved = cs.moved;
  cs.moved = false;
  bool full = moved || cs.gen != c->tree_gen;
  if (moved || cs.g.xmax != (int32_t)c->H - 1 || cs.g.ymax != (int32_t)c->W - 1 ||
      n > 2 * cs.for_n || cs.for_n > 8 * n) {
    const int32_t was[4] = {cs.g.cs, cs.g.P, cs.g.xmax, cs.g.ymax};
    nn_grid_plan(cs.g, c->H, c->W, 2 * n);       // planned ahead of the growth
    cs.for_n = n;
    if (moved || was[0] != cs.g.cs || was[1] != cs.g.P || was[2] != cs.g.xmax || was[3] != cs.g.ymax)
      full = true;                               // (the same cells: the lists stand)
  }
  if (moved) {                                   // (a build leaves the counts zero again)
    HIPCHK(hipMemsetAsync(cs.cnt.p, 0, sizeof(uint32_t) * (size_t)cs.cnt.cap, st));
    HIPCHK(hipMemsetAsync(cs.part.p, 0, sizeof(unsigned long long) * (size_t)cs.part.cap, st));
  }
  g = cs.g;
  g.cnt = cs.cnt.p;
  g.shift = cs.shift.p;
  g.rank = cs.rank.p;
  g.start_old = cs.start[cs.par].p;
  g.items_old = cs.items[cs.par].p;
  g.built_old = cs.built.p + cs.par;
  g.start = cs.start[cs.par ^ 1].p;
  g.items = cs.items[cs.par ^ 1].p;
  g.built_new = cs.built.p + (cs.par ^ 1);
  g.full = full ? 1 : 0;
  g.part = cs.part.p;
  if (++cs.serial == 0) cs.serial = 1;
  g.serial = cs.serial;
  g.err = c->dd_err.p;
  if (far_cap > 0) {
    g.far_n = cs.far_n.p;
    g.far_j = cs.far_j.p;
    g.far_q = cs.far_q.p;
    g.far_min = (uint32_t)c->nn_far_nodes;
  }
  nn_grid_build(st, g, c->txy.p, hi_p, c->n_ub);
  cs.par ^= 1;
  cs.gen = c->tree_gen;
  return TR_OK;
}

// Nearest nodes of qxy[0, B) among the nodes [0, *hi_p) on stream st -> near (dnear: the exact
// squared distances, optional).  m32: the sweep's scratch (nn_scratch(B, plan) floats; unused by
// NN_CELLS).  mid (optional): recorded between the first part (sweep / cell-list build) and the rest.
static int nn_query(tr_ctx* c, NNMode mode, int set, hipStream_t st, const int2* qxy,
                    const int32_t* live, int64_t B, const int64_t* hi_p, const NNPlan& p, float* m32,
                    int64_t* near, double* dnear, double qmax, ResolvePub pub, hipEvent_t mid) {
  if (mode == NN_SWEEP) {
    nn_sweep(st, qxy, B, c->cx, c->cy, c->t4.p, hi_p, p, m32);
    if (mid) HIPCHK(hipEventRecord(mid, st));
    nn_resolve(st, qxy, B, c->cx, c->cy, c->txy.p, hi_p, p, c->d_maxabs.p, qmax, m32, near, dnear, pub);
    return TR_OK;
  }
  NNGrid cg;
  if (int e = cells_build(c, set, st, hi_p, cg, mode == NN_CELLS_FAR_SWEEP ? B : 0)) return e;
  if (mid) HIPCHK(hipEventRecord(mid, st));
  if (mode == NN_CELLS) {
    nn_grid_query(st, cg, qxy, live, B, near, dnear, pub);
    return TR_OK;
  }
  // the far list's samples (their pixels bounded by qmax like every sample's) through the sweep
  nn_grid_query(st, cg, qxy, live, B, near, dnear, ResolvePub(), pub.flag != nullptr);
  nn_sweep(st, cg.far_q, B, c->cx, c->cy, c->t4.p, hi_p, p, m32, cg.far_n);
  nn_resolve(st, cg.far_q, B, c->cx, c->cy, c->txy.p, hi_p, p, c->d_maxabs.p, qmax, m32, near, dnear,
             pub, cg.far_n, cg.far_j);
  return TR_OK;
}

// |q - centre| bound of clipped samples: max(H - cx, cx, W - cy, cy).
static double sample_qmax(const tr_ctx* c) {
  return (double)std::max(std::max(c->H - c->cx, (int64_t)c->cx), std::max(c->W - c->cy, (int64_t)c->cy));
}


static void harvest_side(tr_ctx* c, int ts);

static DDClaim dd_claim_args(const tr_ctx* c) {
  DDClaim d;
  d.btab = c->btab.p;
  d.blast = c->blast.p;
  d.bmask = c->bmask;
  d.epoch = c->epoch;
  d.special = c->dd_special.p;
  d.straight_reject = c->book.straight_reject ? 1 : 0;
  return d;
}



// Look-ahead on the side stream: a future batch's samples and nearest nodes over the tree after
// the latest dedupe.  The batch's own pipe_expand then only sweeps the nodes appended since and
// expands every sample (the expansion's pose-table lookups need the batch's own snapshot).
static int stage_batch(tr_ctx* c, const double* d_gauss, int64_t B, tr_sample* d_samples,
                       tr_record* d_records) {
  if (c->st_n == tr_ctx::SQ) return fail(TR_E_STATE, "look-ahead queue full");
  const int k = c->alloc_k();
  const NNPlan pa = nn_plan(B, c->n_ub);
  if (int e = grow(c, c->s_qxy[k], B)) return e;
  if (int e = grow(c, c->s_live[k], B)) return e;
  if (int e = grow(c, c->s_near[k], B)) return e;
  if (int e = grow(c, c->s_dnear[k], B)) return e;
  const NNMode mode = nn_mode(c, B);
  hipStream_t s = c->side;
  if (mode != NN_CELLS)
    if (int e = grow(c, c->s_m32[k], nn_scratch(B, pa))) return e;
  const int slot = (int)(c->epoch & 3);
  const double qmax = sample_qmax(c);
  double* sp = c->stage_us;                       // TR_TRACE: host time of each call below
  double t0 = c->trace_on ? now_us() : 0.0;
  const double t_in = t0;
  double lp[5] = {0, 0, 0, 0, 0};
  auto lap = [&](int q) { if (c->trace_on) { const double t = now_us(); sp[q] += t - t0; lp[q] = t - t0; t0 = t; } };
  if (c->gate)                                       // the tree after the latest dedupe
    launch_gate(s, c->dd_done.p, c->epoch, c->dd_err.p);
  else
    HIPCHK(hipStreamWaitEvent(s, c->ev_latest, 0));
  lap(0);
  HIPCHK(c->n_chg.reserve(tr_ctx::NS));
  launch_samples(s, c->P, c->G(), d_gauss, B, c->goal[0], c->goal[1], c->goal[2], d_samples,
                 c->s_qxy[k].p, c->s_live[k].p, c->n_chg.p + k);
  // timing level 1 brackets the sweep of every 4th look-ahead only (event records on the side
  // stream cost the pipeline GPU time); level 2 every one
  const int ts = c->ts_next;
  const bool tsamp = c->timing && (c->timing > 1 || (c->stage_seq++ & c->tmask) == 0);
  if (tsamp) {
    if (c->ts_used[ts]) harvest_side(c, ts);
    c->ts_next = (ts + 1) % tr_ctx::TS;
    HIPCHK(hipEventRecord(c->ts_ev[ts][0], s));
  }
  lap(1);
  // (timed as "pass1" / "resolve": the sweep and its resolve, or the cell lists' build and the rest)
  tr_ctx::Stage& q = c->stq[c->st_n];
  ResolvePub pub;                          // gate mode: the last kernel's last block publishes q.seq
  if (c->gate) {
    q.seq = ++c->st_seq;
    pub.flag = c->st_done.p;
    pub.v = q.seq;
    pub.blocks = c->st_blocks.p;
  }
  if (int e = nn_query(c, mode, 1, s, c->s_qxy[k].p, c->s_live[k].p, B, c->snap.p + slot, pa,
                       c->s_m32[k].p, c->s_near[k].p, c->s_dnear[k].p, qmax, pub,
                       tsamp ? c->ts_ev[ts][1] : nullptr))
    return e;
  lap(2);
  if (tsamp) {
    HIPCHK(hipEventRecord(c->ts_ev[ts][2], s));
    c->ts_used[ts] = true;
    c->ts_last = ts;
  }
  lap(3);
  HIPCHK(hipGetLastError());
  if (!c->gate) HIPCHK(hipEventRecord(q.ev, s));
  lap(4);
  if (c->trace_on && c->stage_n++ < 10)      // a run's first look-aheads, call by call
    fprintf(stderr, "stage call %d at %.1f us: gate %.1f samples %.1f nn %.1f timing %.1f rest %.1f\n", c->stage_n,
            t_in - c->trace_t0, lp[0], lp[1], lp[2], lp[3], lp[4]);
  q.gauss = d_gauss;
  q.B = B;
  q.smp = d_samples;
  q.rec = d_records;
  q.k = k;
  q.slot = slot;
  q.plan = pa;
  q.n_lb = c->N;
  q.epoch = c->epoch;
  c->st_n++;
  return TR_OK;
}

// Adds a timed staged sweep's pass1 and resolve durations to the run sums (waits for it).
static void harvest_side(tr_ctx* c, int ts) {
  float a = 0, b = 0;
  if (hipEventSynchronize(c->ts_ev[ts][2]) == hipSuccess &&
      hipEventElapsedTime(&a, c->ts_ev[ts][0], c->ts_ev[ts][1]) == hipSuccess &&
      hipEventElapsedTime(&b, c->ts_ev[ts][1], c->ts_ev[ts][2]) == hipSuccess) {
    c->ts_sum[0] += a * 1e3;
    c->ts_sum[1] += b * 1e3;
    c->ts_n++;
  }
  (void)hipGetLastError();
  c->ts_used[ts] = false;
}

static void harvest_all_side(tr_ctx* c) {
  for (int q = 0; q < tr_ctx::TS; ++q)
    if (c->ts_used[q]) harvest_side(c, q);
}

static void harvest_main(tr_ctx* c, int m) {
  float a = 0, b = 0, d = 0;
  if (hipEventSynchronize(c->tm_ev[m][4]) == hipSuccess &&
      hipEventElapsedTime(&a, c->tm_ev[m][0], c->tm_ev[m][1]) == hipSuccess &&
      hipEventElapsedTime(&b, c->tm_ev[m][1], c->tm_ev[m][2]) == hipSuccess &&
      hipEventElapsedTime(&d, c->tm_ev[m][3], c->tm_ev[m][4]) == hipSuccess) {
    c->tm_sum[0] += a * 1e3;
    c->tm_sum[1] += b * 1e3;
    c->tm_sum[2] += d * 1e3;
    c->tm_n++;
  }
  (void)hipGetLastError();
  c->tm_used[m] = false;
}

static void harvest_all_main(tr_ctx* c) {
  for (int q = 0; q < tr_ctx::TM; ++q)
    if (c->tm_used[q]) harvest_main(c, q);
}

// Fused per-sample pass for B samples against the device tree: rand_conf + freespace, nearest
// node, steer / body rays / drive, arc check (+ goal test).  Async on the context stream.  For a
// staged batch: sweep of the nodes appended since its snapshot, then steer ... arc again only for
// the samples whose nearest node changed.
static int expand_batch(tr_ctx* c, const double* d_gauss, int64_t B, const double* goal3,
                        tr_sample* d_samples, tr_record* d_records) {
  const double qmax = sample_qmax(c);
  const tr_ctx::Stage fr = c->stq[0];
  // a stage is this batch's when its buffers match and its snapshot slot (epoch & 3, a ring of
  // four) has not been reused by later dedupes
  const bool staged = c->st_n > 0 && fr.gauss == d_gauss && fr.B == B && fr.smp == d_samples &&
                      fr.rec == d_records && c->epoch - fr.epoch < 4;
  if (c->st_n > 0 && !staged) {               // stages for other batches: drop them
    HIPCHK(hipStreamSynchronize(c->side));
    c->st_n = 0;
  }
  c->last_staged = staged;
  if (staged) {
    for (int q = 1; q < c->st_n; ++q) std::swap(c->stq[q - 1], c->stq[q]);   // pop (events kept)
    c->st_n--;
    const int k = fr.k;
    int2* qxy = c->s_qxy[k].p;
    if (int e = grow(c, c->chg, B)) return e;
    int32_t* nchg = c->n_chg.p + k;             // zeroed by the stage's sample kernel
    if (c->gate) {
      if (c->gated_seq != fr.seq)            // the last k_dd did not already wait for it
        launch_gate(c->st, c->st_done.p, fr.seq, c->dd_err.p);
    } else {
      HIPCHK(hipStreamWaitEvent(c->st, fr.ev, 0));
    }
    if (c->timing > 1) HIPCHK(hipEventRecord(c->t_ev[0], c->st));
    int ms = -1;                                // sampled main-stream timing (level 1)
    if (c->timing == 1 && c->tm_pending < 0 && (c->main_seq++ & c->tmask) == 0) {
      ms = c->tm_next;
      if (c->tm_used[ms]) harvest_main(c, ms);
      c->tm_next = (ms + 1) % tr_ctx::TM;
      HIPCHK(hipEventRecord(c->tm_ev[ms][0], c->st));
    }
    // the correction by the nodes appended since the look-ahead's snapshot: inside the expansion
    // kernel (default) or as its own kernel (TR_FUSED_DELTA=0; the timings then split them)
    DeltaArgs da;
    if (c->fused_delta) {
      da.snap = c->snap.p + fr.slot;
      da.count = c->d_count.p;
      da.dnear = c->s_dnear[k].p;
      da.t4 = c->t4.p;
      da.maxabs = c->d_maxabs.p;
      da.qmax = qmax;
      da.cx = c->cx;
      da.cy = c->cy;
      bool binned = c->delta_bins && c->db_cnt.p;   // every dedupe since the look-ahead binned
      for (unsigned long long e = fr.epoch + 1; binned && e <= c->epoch; ++e) binned = c->db_ok[e & 3] == e;
      da.e_lo = fr.epoch + 1;
      da.e_hi = c->epoch;
      if (binned) da.bins = c->bins_view();
    } else {
      nn_delta(c->st, qxy, B, c->txy.p, c->snap.p + fr.slot, c->d_count.p, c->s_live[k].p,
               c->s_near[k].p, c->s_dnear[k].p, c->chg.p, nchg);
    }
    if (c->timing > 1) HIPCHK(hipEventRecord(c->t_ev[1], c->st));
    if (ms >= 0) HIPCHK(hipEventRecord(c->tm_ev[ms][1], c->st));
    // every sample against its corrected nearest node (+ the snapshot lookups of the dedupe)
    launch_expand_arc(c->st, c->P, c->G(), c->s_near[k].p, B, d_samples, c->s_live[k].p, c->txy.p,
                      c->tth.p, goal3[0], goal3[1], goal3[2], c->htab.p, c->hmask, c->dd_err.p,
                      d_records, da);
    if (ms >= 0) {
      HIPCHK(hipEventRecord(c->tm_ev[ms][2], c->st));
      c->tm_pending = ms;                       // the batch's dedupe records [3], [4]
    }
    if (c->timing > 1) {             // [2] steer ... arc (one kernel), [3] = [2]
      HIPCHK(hipEventRecord(c->t_ev[2], c->st));
      HIPCHK(hipEventRecord(c->t_ev[3], c->st));
    }
    HIPCHK(hipGetLastError());
    return TR_OK;
  }
  const int k = c->alloc_k();
  const NNPlan p = nn_plan(B, c->n_ub);
  if (int e = grow(c, c->s_qxy[k], B)) return e;
  if (int e = grow(c, c->s_live[k], B)) return e;
  if (int e = grow(c, c->s_near[k], B)) return e;
  const NNMode mode = nn_mode(c, B);
  if (mode != NN_CELLS)
    if (int e = grow(c, c->s_m32[k], nn_scratch(B, p))) return e;
  int2* qxy = c->s_qxy[k].p;
  int32_t* live = c->s_live[k].p;
  launch_samples(c->st, c->P, c->G(), d_gauss, B, goal3[0], goal3[1], goal3[2], d_samples, qxy, live);
  if (c->timing) HIPCHK(hipEventRecord(c->t_ev[0], c->st));
  if (int e = nn_query(c, mode, 0, c->st, qxy, live, B, c->d_count.p, p, c->s_m32[k].p,
                       c->s_near[k].p, nullptr, qmax, ResolvePub(), nullptr))
    return e;
  if (c->timing) HIPCHK(hipEventRecord(c->t_ev[1], c->st));
  launch_expand_arc(c->st, c->P, c->G(), c->s_near[k].p, B, d_samples, live, c->txy.p, c->tth.p,
                    goal3[0], goal3[1], goal3[2], c->htab.p, c->hmask, c->dd_err.p, d_records);
  if (c->timing > 1) {
    HIPCHK(hipEventRecord(c->t_ev[2], c->st));
    HIPCHK(hipEventRecord(c->t_ev[3], c->st));
  }
  HIPCHK(hipGetLastError());
  return TR_OK;
}

// ------------------------------------------------------------------ device gaussian stream
static int64_t rng_words(int64_t n) { return 4 * rng_attempts_ub(n); }

// Ring for chunks of up to n gaussians: two chunks' worth of words ahead of the current position
// plus the blocks a rewind / get_state may still need.  Growth keeps the live window [block of the
// current position, words generated).
static int rng_ensure(tr_ctx* c, int64_t n) {
  if (!c->rng_on) return fail(TR_E_STATE, "no gaussian stream: call tr_rng_set_state");
  const int64_t need = ((2 * rng_words(n) + rng_ring_extra(n) + 3 * 624 + 623) / 624) * 624;
  HIPCHK(c->rng_cnt.reserve(rng_counts_len(n)));
  if (need <= c->rng_rs) return TR_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->rng_st));
  RngPos p;
  int64_t gen[2] = {0, 0};
  HIPCHK(copy_sync(c->st, &p, c->rng_pos.p, sizeof(p), hipMemcpyDeviceToHost));
  HIPCHK(copy_sync(c->st, gen, c->rng_gen.p, sizeof(gen), hipMemcpyDeviceToHost));
  const int64_t ge = gen[0];
  // everything the old ring holds moves over (the current position's block, and the history a
  // jump-ahead reads); the oldest word kept is recorded for the generator
  const int64_t b0 = std::max(gen[1], std::max<int64_t>(0, ge - c->rng_rs));
  std::vector<uint32_t> live((size_t)(ge - b0));
  for (int64_t w = b0; w < ge; w += 624)
    HIPCHK(copy_sync(c->st, live.data() + (w - b0), c->rng_ring.p + w % c->rng_rs, 624 * 4, hipMemcpyDeviceToHost));
  c->rng_ring.release();
  HIPCHK(c->rng_ring.reserve(need));
  c->rng_rs = need;
  for (int64_t w = b0; w < ge; w += 624)
    HIPCHK(copy_sync(c->st, c->rng_ring.p + w % need, live.data() + (w - b0), 624 * 4, hipMemcpyHostToDevice));
  HIPCHK(copy_sync(c->st, c->rng_gen.p + 1, &b0, sizeof(b0), hipMemcpyHostToDevice));
  return TR_OK;
}

static int rng_check(tr_ctx* c) {
  int32_t e = 0;
  HIPCHK(copy_sync(c->st, &e, c->rng_err.p, 4, hipMemcpyDeviceToHost));
  if (e) return fail(TR_E_STATE, "gaussian stream: the word ring ran short of a chunk (bound broken; bits " +
                                     std::to_string(e) + ")");
  return TR_OK;
}

// Stream gates need the device to run kernels of two streams at the same time: a gate kernel spins
// until a kernel of the other stream has stored a flag.  A tool that serializes every dispatch
// (counter collection: rocprofv3 --pmc) would leave the gate waiting for a kernel that cannot
// start.  Two one-wave kernels, one per stream, each store their own flag and wait (20 ms at most)
// for the other's: both see it only when they were running together.
static int gate_probe(tr_ctx* c, bool* concurrent) {
  DBuf<unsigned long long> f;
  HIPCHK(f.reserve(4));
  HIPCHK(fill_sync(c->own, f.p, 0, 4 * sizeof(unsigned long long)));
  launch_handshake(c->own, f.p, f.p + 1, 2000000ull, f.p + 2);
  launch_handshake(c->side, f.p + 1, f.p, 2000000ull, f.p + 3);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->own));
  HIPCHK(hipStreamSynchronize(c->side));
  unsigned long long ok[2] = {0, 0};
  HIPCHK(copy_sync(c->own, ok, f.p + 2, sizeof(ok), hipMemcpyDeviceToHost));
  *concurrent = ok[0] && ok[1];
  f.release();
  return TR_OK;
}

extern "C" {

const char* tr_last_error(void) { return g_err.c_str(); }

int tr_set_option(tr_ctx* c, const char* name, int64_t value) {
  if (!c || !name) return fail(TR_E_ARG, "NULL argument");
  if (c->r_count || c->st_n) return fail(TR_E_STATE, "set_option with batches in flight");
  const std::string k(name);
  if (k == "gate") {
    if (set_dev(c)) return TR_E_HIP;
    HIPCHK(hipStreamSynchronize(c->st));
    HIPCHK(hipStreamSynchronize(c->side));
    c->gate = value != 0;
    if (c->gate && c->dd_done.p) {     // the flags name the points both streams have reached
      const unsigned long long ep = c->epoch, sq = c->st_seq;
      HIPCHK(copy_sync(c->st, c->dd_done.p, &ep, sizeof(ep), hipMemcpyHostToDevice));
      HIPCHK(copy_sync(c->st, c->st_done.p, &sq, sizeof(sq), hipMemcpyHostToDevice));
    }
  } else if (k == "fused_delta") {
    c->fused_delta = value != 0;
  } else if (k == "delta_bins") {
    c->delta_bins = value != 0;
  } else if (k == "nn_grid") {
    c->nn_grid = value != 0;
  } else if (k == "nn_far_sweep") {
    if (value < 0) return fail(TR_E_ARG, "nn_far_sweep < 0");
    c->nn_far_sweep = value;
  } else if (k == "nn_far_nodes") {
    if (value < 0 || value > INT32_MAX) return fail(TR_E_ARG, "nn_far_nodes out of range");
    c->nn_far_nodes = value;
  } else if (k == "nn_grid_min") {
    c->nn_grid_min = value;
  } else if (k == "dd_fused") {
    c->dd_fused = value != 0;
  } else if (k == "dd_gatefold") {
    c->dd_gatefold = value != 0;
  } else if (k == "dd_fused_max") {
    if (value < 0) return fail(TR_E_ARG, "dd_fused_max < 0");
    c->dd_fused_max = value;
  } else if (k == "book") {
    std::lock_guard<std::mutex> lk(c->mu);
    c->replay_on = value != 0;
  } else if (k == "trace") {
    c->trace_on = value != 0;
  } else {
    return fail(TR_E_ARG, "unknown option '" + k + "'");
  }
  return TR_OK;
}

int tr_get_option(const tr_ctx* c, const char* name, int64_t* value) {
  if (!c || !name || !value) return fail(TR_E_ARG, "NULL argument");
  const std::string k(name);
  if (k == "gate") *value = c->gate;
  else if (k == "fused_delta") *value = c->fused_delta;
  else if (k == "delta_bins") *value = c->delta_bins;
  else if (k == "head_waits") *value = (int64_t)c->head_waits.load();
  else if (k == "nn_grid") *value = c->nn_grid;
  else if (k == "nn_far_sweep") *value = c->nn_far_sweep;
  else if (k == "nn_far_nodes") *value = c->nn_far_nodes;
  else if (k == "nn_grid_min") *value = c->nn_grid_min;
  else if (k == "dd_fused") *value = c->dd_fused;
  else if (k == "dd_gatefold") *value = c->dd_gatefold;
  else if (k == "dd_fused_max") *value = c->dd_fused_max;
  else if (k == "book") *value = c->replay_on;
  else if (k == "trace") *value = c->trace_on;
  else return fail(TR_E_ARG, "unknown option '" + k + "'");
  return TR_OK;
}
int tr_version(void) { return 3; }

int tr_create(int device, tr_ctx** out) {
  if (!out) return fail(TR_E_ARG, "out is NULL");
  GUARD({
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(TR_E_ARG, "no such HIP device");
    std::unique_ptr<tr_ctx> c(new tr_ctx());
    c->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    c->st = c->own;
    for (auto& e : c->t_ev) HIPCHK(hipEventCreate(&e));
    for (auto& e : c->r_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& b : c->r_cr) b.flags = hipHostMallocCoherent | hipHostMallocMapped;
    c->r_ready.flags = hipHostMallocCoherent | hipHostMallocMapped;
    HIPCHK(c->r_ready.reserve(tr_ctx::R));
    for (int k = 0; k < tr_ctx::R; ++k) c->r_ready.p[k] = 0;
    HIPCHK(c->err.reserve(4));
    HIPCHK(c->d_count.reserve(1));
    HIPCHK(c->d_maxabs.reserve(1));
    HIPCHK(c->snap.reserve(4));
    HIPCHK(c->dd_err.reserve(1));
    HIPCHK(fill_sync(c->st, c->dd_err.p, 0, sizeof(int32_t)));
    HIPCHK(c->st_done.reserve(1));
    HIPCHK(fill_sync(c->st, c->st_done.p, 0, sizeof(unsigned long long)));
    HIPCHK(c->st_blocks.reserve(1));
    HIPCHK(fill_sync(c->st, c->st_blocks.p, 0, sizeof(int32_t)));
    // every stream at the default priority (streams of different priorities have hung this pool)
    HIPCHK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    // cross-stream edges in event mode (look-ahead <-> batch): the look-ahead waits on its own
    // dedupe event ev_dd, not on the commit event r_ev[k]: the replay worker blocks in
    // hipEventSynchronize on r_ev[k], which holds that event's lock until the batch completes, and
    // a hipStreamWaitEvent on the same event then stalls the enqueue thread (~17 us per batch).
    HIPCHK(hipEventCreateWithFlags(&c->ev_dd, hipEventDisableTiming));
    for (auto& q : c->stq) HIPCHK(hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
    for (auto& tri : c->ts_ev)
      for (auto& e : tri) HIPCHK(hipEventCreate(&e));
    for (auto& five : c->tm_ev)
      for (auto& e : five) HIPCHK(hipEventCreate(&e));
    HIPCHK(fill_sync(c->st, c->snap.p, 0, 4 * sizeof(int64_t)));
    HIPCHK(fill_sync(c->st, c->d_count.p, 0, sizeof(int64_t)));
    HIPCHK(fill_sync(c->st, c->d_maxabs.p, 0, sizeof(unsigned long long)));
    HIPCHK(hipStreamCreateWithFlags(&c->rng_st, hipStreamNonBlocking));
    for (auto& e : c->rng_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->rng_free, hipEventDisableTiming));
    for (auto& e : c->rng_b) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(c->rng_err_h.reserve(1));
    HIPCHK(c->rng_pos.reserve(2 + 8 * tr_ctx::RC));
    HIPCHK(c->rng_keys.reserve(624 * 8 * tr_ctx::RC));
    HIPCHK(c->rng_gen.reserve(2));
    HIPCHK(c->rng_err.reserve(1));
    HIPCHK(fill_sync(c->st, c->rng_err.p, 0, sizeof(int32_t)));
    HIPCHK(c->rng_done.reserve(1));
    HIPCHK(c->rng_flag.reserve(1));
    HIPCHK(fill_sync(c->st, c->rng_flag.p, 0, sizeof(unsigned long long)));
    HIPCHK(fill_sync(c->st, c->rng_done.p, 0, sizeof(int32_t)));
    HIPCHK(c->rng_seeds.reserve(16 * 624));
    if (int e = scratch_resolve(device)) return e;
    bool concurrent = true;
    if (int e = gate_probe(c.get(), &concurrent)) return e;
    // Streams past the device's hardware queues share them, and two streams on one queue run one
    // after the other: a few more candidates for the look-ahead stream before settling for event
    // edges (under a serializing profiler every one of them fails the probe).
    std::vector<hipStream_t> spare;
    for (int tries = 0; !concurrent && tries < 3; ++tries) {
      hipStream_t s2 = nullptr;
      HIPCHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      spare.push_back(c->side);
      c->side = s2;
      if (int e = gate_probe(c.get(), &concurrent)) return e;
    }
    for (hipStream_t q : spare) (void)hipStreamDestroy(q);
    c->gate = concurrent;              // else event edges (tr_get_option "gate" reports it)
    // main.py:14-32 defaults
    c->P = Params{5, -65, 65, 2, 30, .6, .4, 100, 10, 45, 1, 0};
    *out = c.release();
    return TR_OK;
  })
}

int tr_destroy(tr_ctx* c) {
  if (!c) return TR_OK;
  worker_stop(c);
  if (c->comm) {
    (void)hipStreamSynchronize(c->st);
    rccl()->destroy(c->comm);
  }
  (void)hipSetDevice(c->device);
  if (c->st) (void)hipStreamSynchronize(c->st);
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (int k = 0; k < tr_ctx::NS; ++k) {
    c->s_qxy[k].release(); c->s_live[k].release(); c->s_m32[k].release();
    c->s_near[k].release(); c->s_dnear[k].release();
  }
  c->chg.release(); c->n_chg.release();
  c->snap.release();
  for (auto& cs : c->cells) {
    cs.cnt.release(); cs.shift.release(); cs.rank.release(); cs.built.release(); cs.part.release();
    cs.far_n.release(); cs.far_j.release(); cs.far_q.release();
    for (int q = 0; q < 2; ++q) { cs.start[q].release(); cs.items[q].release(); }
  }
  c->db_cnt.release(); c->db_items.release(); c->db_ovf.release();
  if (c->ev_dd) (void)hipEventDestroy(c->ev_dd);
  for (auto& q : c->stq)
    if (q.ev) (void)hipEventDestroy(q.ev);
  for (auto& tri : c->ts_ev)
    for (hipEvent_t e : tri)
      if (e) (void)hipEventDestroy(e);
  for (auto& five : c->tm_ev)
    for (hipEvent_t e : five)
      if (e) (void)hipEventDestroy(e);
  if (c->side) (void)hipStreamDestroy(c->side);

  if (c->rng_st) {
    (void)hipStreamSynchronize(c->rng_st);
    (void)hipStreamDestroy(c->rng_st);
  }
  for (auto& e : c->rng_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->rng_free) (void)hipEventDestroy(c->rng_free);
  for (auto& e : c->rng_b)
    if (e) (void)hipEventDestroy(e);
  c->rng_err_h.release();
  c->rng_ring.release(); c->rng_gen.release(); c->rng_pos.release(); c->rng_cnt.release();
  c->rng_err.release(); c->rng_out.release(); c->rng_keys.release();
  c->rng_done.release(); c->rng_seeds.release(); c->rng_flag.release();
  c->hg_send.release(); c->hg_recv.release();
  c->grid.release(); c->txy.release(); c->t4.release(); c->tth.release();
  c->d_count.release(); c->d_maxabs.release(); c->htab.release(); c->btab.release();
  c->blast.release(); c->dd_base.release(); c->dd_special.release();
  c->dd_done.release(); c->dd_blocks.release(); c->st_done.release(); c->st_blocks.release();
  DBuf<int32_t>* v[4] = {&c->dd_slot, &c->dd_lr, &c->live, &c->err};
  for (auto* b : v) b->release();
  c->dd_bc.release(); c->dd_err.release(); c->dd_ticket.release(); c->dd_bst.release(); c->dd_idx.release();
  c->qxy.release(); c->m32.release(); c->iout.release(); c->cnt.release(); c->samp.release();
  c->rec.release(); c->rec_all.release(); c->gauss.release(); c->fin.release(); c->fout.release(); c->bout.release();
  c->i32.release(); c->h_x.release();
  c->fn_par.release(); c->fn_child.release(); c->fn_out.release();
  c->fn_pose.release(); c->fn_goal.release(); c->fn_d.release(); c->fn_part.release();
  c->as_work.release(); c->as_sg.release(); c->as_path.release(); c->as_len.release(); c->as_stats.release();
  for (int k = 0; k < tr_ctx::R; ++k) {
    c->r_cr[k].release();
    if (c->r_ev[k]) (void)hipEventDestroy(c->r_ev[k]);
  }
  c->r_ready.release();
  for (auto& e : c->t_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  return TR_OK;
}

int tr_set_stream(tr_ctx* c, void* s) {
  if (!c) return fail(TR_E_ARG, "ctx is NULL");
  const hipStream_t to = s ? (hipStream_t)s : c->own;
  if (to != c->st) {                // the device tree and cell lists are ordered by the stream
    if (set_dev(c)) return TR_E_HIP;
    HIPCHK(hipStreamSynchronize(c->st));
  }
  c->st = to;
  return TR_OK;
}

int tr_sync(tr_ctx* c) {
  if (!c) return fail(TR_E_ARG, "ctx is NULL");
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->side));
  return TR_OK;
}

int tr_set_params(tr_ctx* c, const tr_params* p) {
  if (!c || !p) return fail(TR_E_ARG, "NULL argument");
  if (c->r_count || c->st_n) return fail(TR_E_STATE, "set_params with batches in flight");
  c->P = Params{p->bikelength, p->leftconstraint, p->rightconstraint, p->frontclearance,
                p->maxdrivedist, p->weightxy, p->xystdv, p->anglestdv, p->tol_xy, p->tol_ang,
                p->forwardonly, 0};
  std::lock_guard<std::mutex> lk(c->mu);    // the replay worker reads it
  c->book.straight_reject = p->straight_reject != 0;
  return TR_OK;
}

int tr_set_grid(tr_ctx* c, const uint8_t* free_yx, int64_t H, int64_t W) {
  if (!c || !free_yx || H <= 0 || W <= 0) return fail(TR_E_ARG, "bad grid");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->side));
  // main.py:37-42's bool array, one bit per cell (geom.hpp Grid): packed here, kept on both sides
  GUARD({
    const int64_t wpr = (W + 31) / 32;
    c->hbits.assign((size_t)grid_words(H, W), 0u);
    for (int64_t y = 0; y < H; ++y) {
      const uint8_t* row = free_yx + y * W;
      uint32_t* out = c->hbits.data() + y * wpr;
      for (int64_t x = 0; x < W; ++x)
        if (row[x]) out[x >> 5] |= 1u << (x & 31);
    }
    c->hgrid.assign(free_yx, free_yx + H * W);
  })
  HIPCHK(c->grid.reserve((int64_t)c->hbits.size()));
  HIPCHK(copy_sync(c->st, c->grid.p, c->hbits.data(), sizeof(uint32_t) * c->hbits.size(),
                   hipMemcpyHostToDevice));
  c->H = H;
  c->W = W;
  c->have_grid = true;
  return TR_OK;
}

int tr_tree_reset(tr_ctx* c, int64_t cap) {
  if (!c || cap < 0) return fail(TR_E_ARG, "bad capacity");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->side));
  c->st_n = 0;
  c->N = c->n_ub = 0;
  c->tree_gen++;
  c->cx = c->have_grid ? (int32_t)(c->H / 2) : 0;   // x indexes shape[0] (search.py:17-23)
  c->cy = c->have_grid ? (int32_t)(c->W / 2) : 0;
  HIPCHK(fill_sync(c->st, c->snap.p, 0, 4 * sizeof(int64_t)));
  HIPCHK(fill_sync(c->st, c->d_count.p, 0, sizeof(int64_t)));
  HIPCHK(fill_sync(c->st, c->d_maxabs.p, 0, sizeof(unsigned long long)));
  if (int e = ensure_tree(c, std::max<int64_t>(cap, 1))) return e;
  if (int e = ensure_table(c, std::max<int64_t>(cap, 1))) return e;
  HIPCHK(fill_sync(c->st, c->htab.p, 0xff, sizeof(PoseSlot) * (c->hmask + 1)));
  return TR_OK;
}

// Append host poses: the device tree, its fp32 copy, the pose table, count and coordinate bound.
int tr_tree_append(tr_ctx* c, const double* xyt, int64_t n) {
  if (!c || (n && !xyt) || n < 0) return fail(TR_E_ARG, "bad tree append");
  if (!n) return TR_OK;
  if (set_dev(c)) return TR_E_HIP;
  if (c->r_count || c->st_n) return fail(TR_E_STATE, "tree append while batches are in flight");
  GUARD({
    HIPCHK(hipStreamSynchronize(c->st));
    if (int e = ensure_tree(c, c->N + n)) return e;
    HIPCHK(c->h_x.reserve(5 * n + 2));
    double* hx = c->h_x.p;
    float4* f = reinterpret_cast<float4*>(hx + ((3 * n + 1) & ~(int64_t)1));   // 16 B aligned
    unsigned long long mb = 0;
    HIPCHK(copy_sync(c->st, &mb, c->d_maxabs.p, sizeof(mb), hipMemcpyDeviceToHost));
    double mx;
    memcpy(&mx, &mb, 8);
    for (int64_t i = 0; i < n; ++i) {
      const double x = xyt[3 * i], y = xyt[3 * i + 1];
      hx[2 * i] = x;
      hx[2 * i + 1] = y;
      hx[2 * n + i] = xyt[3 * i + 2];
      f[i] = screen_node(x, y, c->cx, c->cy);
      mx = std::max(mx, centred_abs(x, y, c->cx, c->cy));
    }
    memcpy(&mb, &mx, 8);
    HIPCHK(copy_sync(c->st, c->txy.p + c->N, hx, sizeof(double2) * n, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(c->st, c->tth.p + c->N, hx + 2 * n, sizeof(double) * n, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(c->st, c->t4.p + c->N, f, sizeof(float4) * n, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(c->st, c->d_maxabs.p, &mb, sizeof(mb), hipMemcpyHostToDevice));
    c->N += n;
    c->n_ub = c->N;
    HIPCHK(copy_sync(c->st, c->d_count.p, &c->N, sizeof(int64_t), hipMemcpyHostToDevice));
    HIPCHK(copy_sync(c->st, c->snap.p + (c->epoch & 3), &c->N, sizeof(int64_t), hipMemcpyHostToDevice));
    if (int e = ensure_table(c, c->N)) return e;
    dd_rebuild(c->st, c->htab.p, c->hmask, c->dd_err.p, c->txy.p, c->tth.p, c->N);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    return TR_OK;
  })
}

int64_t tr_tree_size(const tr_ctx* c) { return c ? c->N : -1; }

int tr_nn_batch(tr_ctx* c, const int32_t* q_xy, int64_t B, int64_t* out_idx, double* out_d2) {
  if (!c || B < 0 || (B && (!q_xy || !out_idx))) return fail(TR_E_ARG, "bad nn batch");
  if (!B) return TR_OK;
  if (c->N <= 0) return fail(TR_E_STATE, "empty tree");
  if (set_dev(c)) return TR_E_HIP;
  double qmax = 0;
  for (int64_t j = 0; j < B; ++j)
    qmax = std::max(qmax, centred_abs((double)q_xy[2 * j], (double)q_xy[2 * j + 1], c->cx, c->cy));
  const NNMode mode = nn_mode(c, B);
  const NNPlan p = nn_plan(B, c->n_ub);
  if (mode != NN_CELLS) HIPCHK(c->m32.reserve(nn_scratch(B, p)));
  HIPCHK(c->qxy.reserve(B));
  HIPCHK(c->iout.reserve(B));
  HIPCHK(c->fout.reserve(B));
  HIPCHK(hipMemcpyAsync(c->qxy.p, q_xy, sizeof(int32_t) * 2 * B, hipMemcpyHostToDevice, c->st));
  if (int e = nn_query(c, mode, 0, c->st, c->qxy.p, nullptr, B, c->d_count.p, p, c->m32.p, c->iout.p,
                       c->fout.p, qmax, ResolvePub(), nullptr))
    return e;
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out_idx, c->iout.p, sizeof(int64_t) * B, hipMemcpyDeviceToHost, c->st));
  if (out_d2)
    HIPCHK(hipMemcpyAsync(out_d2, c->fout.p, sizeof(double) * B, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return TR_OK;
}

int tr_los_batch(tr_ctx* c, const double* seg4, int64_t n, uint8_t* out) {
  if (int e = need_grid(c)) return e;
  if (n < 0 || (n && (!seg4 || !out))) return fail(TR_E_ARG, "bad los batch");
  if (!n) return TR_OK;
  HIPCHK(c->fin.reserve(4 * n));
  HIPCHK(c->bout.reserve(n));
  HIPCHK(hipMemsetAsync(c->err.p, 0, 4, c->st));
  HIPCHK(hipMemcpyAsync(c->fin.p, seg4, sizeof(double) * 4 * n, hipMemcpyHostToDevice, c->st));
  launch_los_f64(c->st, c->G(), c->fin.p, n, c->bout.p, c->err.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->bout.p, n, hipMemcpyDeviceToHost, c->st));
  return check_err_word(c);
}

int tr_los_batch_dev(tr_ctx* c, const int32_t* d_seg4, int64_t n, uint8_t* d_out) {
  if (int e = need_grid(c)) return e;
  if (n < 0 || (n && (!d_seg4 || !d_out))) return fail(TR_E_ARG, "bad los batch");
  if (!n) return TR_OK;
  launch_los_i32(c->st, c->G(), d_seg4, n, d_out, c->err.p);
  HIPCHK(hipGetLastError());
  return TR_OK;
}

// findnearest over E edges: poses already on the device (xs/ys/ths with strides), edges and goals
// from the host; results copied back, synchronous.
static int findnearest_dev(tr_ctx* c, const double* xs, int sx, const double* ys, int sy,
                           const double* ths, int sth, const int64_t* e_par,
                           const int64_t* e_child, int64_t E, const double* goals3, int64_t G,
                           int64_t* out_child, double* out_dist) {
  HIPCHK(c->fn_par.reserve(std::max<int64_t>(E, 1)));
  HIPCHK(c->fn_child.reserve(std::max<int64_t>(E, 1)));
  HIPCHK(c->fn_goal.reserve(3 * G));
  HIPCHK(c->fn_out.reserve(G));
  HIPCHK(c->fn_d.reserve(G));
  HIPCHK(c->fn_part.reserve(fn_scratch(E, G)));
  if (E) {
    HIPCHK(hipMemcpyAsync(c->fn_par.p, e_par, sizeof(int64_t) * E, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->fn_child.p, e_child, sizeof(int64_t) * E, hipMemcpyHostToDevice, c->st));
  }
  HIPCHK(hipMemcpyAsync(c->fn_goal.p, goals3, sizeof(double) * 3 * G, hipMemcpyHostToDevice, c->st));
  launch_findnearest(c->st, xs, sx, ys, sy, ths, sth, c->fn_par.p, c->fn_child.p, E, c->fn_goal.p,
                     G, c->P.weightxy, c->fn_part.p, c->fn_out.p, c->fn_d.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out_child, c->fn_out.p, sizeof(int64_t) * G, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(out_dist, c->fn_d.p, sizeof(double) * G, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return TR_OK;
}

int tr_findnearest_batch(tr_ctx* c, const double* xyt, int64_t n, const int64_t* e_par,
                         const int64_t* e_child, int64_t E, const double* goals3, int64_t G,
                         int64_t* out_child, double* out_dist) {
  if (!c || n < 0 || E < 0 || G < 0 || (n && !xyt) || (E && (!e_par || !e_child)) ||
      (G && (!goals3 || !out_child || !out_dist)))
    return fail(TR_E_ARG, "bad findnearest batch");
  if (G > 65535) return fail(TR_E_ARG, "findnearest: at most 65535 goals per call");
  if (!G) return TR_OK;
  for (int64_t k = 0; k < E; ++k)            // indices are checked here, not on the device
    if (e_child[k] < 0 || e_child[k] >= n || e_par[k] < 0 || e_par[k] >= n)
      return fail(TR_E_ARG, "findnearest: edge " + std::to_string(k) + " out of range");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(c->fn_pose.reserve(std::max<int64_t>(3 * n, 3)));
  if (n)
    HIPCHK(hipMemcpyAsync(c->fn_pose.p, xyt, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->st));
  const double* p = c->fn_pose.p;
  return findnearest_dev(c, p, 3, p + 1, 3, p + 2, 3, e_par, e_child, E, goals3, G, out_child,
                         out_dist);
}

int tr_rrt_findnearest(tr_ctx* c, const double* goals3, int64_t G, int64_t* out_node,
                       double* out_dist) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (c->r_count) return fail(TR_E_STATE, "findnearest: batches still to commit");
  if (!c->replay_on) return fail(TR_E_STATE, "findnearest: this context keeps no book (option book = 0)");
  if (G < 0 || (G && (!goals3 || !out_node || !out_dist))) return fail(TR_E_ARG, "bad findnearest");
  if (G > 65535) return fail(TR_E_ARG, "findnearest: at most 65535 goals per call");
  if (!G) return TR_OK;
  if (set_dev(c)) return TR_E_HIP;
  worker_drain(c);
  HIPCHK(hipStreamSynchronize(c->st));       // the device tree holds every committed node
  const tr_book& b = c->book;
  const double* txy = reinterpret_cast<const double*>(c->txy.p);
  return findnearest_dev(c, txy, 2, txy + 1, 2, c->tth.p, 1, b.e_par.data(), b.e_child.data(),
                         (int64_t)b.e_par.size(), goals3, G, out_node, out_dist);
}

int tr_lineofsight(tr_ctx* c, const double* seg4, uint8_t* out) {
  if (!c || !seg4 || !out) return fail(TR_E_ARG, "NULL argument");
  if (!c->have_grid) return fail(TR_E_STATE, "no grid: call tr_set_grid first");
  const Grid g = c->HG();
  int ierr = 0;
  const bool clear = los(g, V2{seg4[0], seg4[1]}, V2{seg4[2], seg4[3]}, &ierr);
  if (ierr) return fail(TR_E_INDEX, "index is out of bounds (imarray[y][x], search.py:30)");
  *out = clear ? 1 : 0;
  return TR_OK;
}

int tr_astar(tr_ctx* c, int64_t sx, int64_t sy, int64_t gx, int64_t gy, int thetastar,
             int64_t* path_xy, int64_t cap, int64_t* path_len, int64_t* stats4) {
  if (int e = need_grid(c)) return e;
  if (!path_len || !stats4 || cap < 0 || (cap && !path_xy)) return fail(TR_E_ARG, "bad astar arguments");
  GUARD({
    // each popped pair's line of sight on the host (the grid's host copy, the same closed-form
    // Bresenham as the kernels): the serial search never waits for the GPU
    const Grid g = c->HG();
    LosFn host_los = [&g](int64_t x0, int64_t y0, int64_t x1, int64_t y1, bool* clear) -> int {
      int ierr = 0;
      *clear = los_i(g, x0, y0, x1, y1, &ierr);
      if (ierr) return fail(TR_E_INDEX, "index is out of bounds (imarray[y][x], search.py:30)");
      return TR_OK;
    };
    std::vector<int64_t> path;
    AStarStats st;
    std::string msg;
    const int rc = astar_run(c->hgrid.data(), c->H, c->W, sx, sy, gx, gy, thetastar != 0, host_los,
                             path, st, msg);
    if (rc) return msg.empty() ? rc : fail(rc, msg);
    stats4[0] = st.expanded;
    stats4[1] = 0;
    stats4[2] = st.los_segments;
    stats4[3] = st.status;
    *path_len = (int64_t)path.size() / 2;
    if (*path_len > cap) return fail(TR_E_ARG, "astar: path longer than cap");
    if (!path.empty()) memcpy(path_xy, path.data(), sizeof(int64_t) * path.size());
    return TR_OK;
  })
}

int tr_astar_batch(tr_ctx* c, const int32_t* sg4, int64_t n, int thetastar, int64_t* path_xy,
                   int64_t cap, int64_t* path_len, int64_t* stats4) {
  if (int e = need_grid(c)) return e;
  if (n < 0 || cap < 0 || (n && (!sg4 || !path_len || !stats4 || (cap && !path_xy))))
    return fail(TR_E_ARG, "bad astar batch");
  if (!n) return TR_OK;
  if (c->H > 65535 || c->W > 65535) return fail(TR_E_ARG, "astar batch: grid sides up to 65535");
  if (c->H * c->W >= (1ll << 30)) return fail(TR_E_ARG, "astar batch: at most 2^30 cells");
  GUARD({
    // per query: the queue's buckets and far list, gScore and state words for every cell; as many
    // queries per launch as fit the work buffer (one wave each)
    const int64_t far_cap = c->H * c->W + 4096;
    const int64_t per = astar_dev_bytes_per_query(c->H, c->W, far_cap);
    const int64_t budget = 96ll << 30;
    const int64_t chunk = std::max<int64_t>(1, std::min(n, budget / per));
    // the work buffers stay with the context (a hipMalloc of tens of GB per call costs more than
    // the search)
    DBuf<uint8_t>& work = c->as_work;
    DBuf<int32_t>& d_sg = c->as_sg;
    DBuf<int64_t>&d_path = c->as_path, &d_len = c->as_len, &d_stats = c->as_stats;
    auto cleanup = [&]() {};
    HIPCHK(hipStreamSynchronize(c->st));
    hipError_t he = work.reserve(per * chunk);
    if (he == hipSuccess) he = d_sg.reserve(4 * chunk);
    if (he == hipSuccess) he = d_path.reserve(std::max<int64_t>(2 * cap * chunk, 1));
    if (he == hipSuccess) he = d_len.reserve(chunk);
    if (he == hipSuccess) he = d_stats.reserve(4 * chunk);
    if (he != hipSuccess)
      return fail(TR_E_HIP, std::string("astar batch: device allocation: ") + hipGetErrorString(he));
    int rc = TR_OK;
    for (int64_t q0 = 0; q0 < n && rc == TR_OK; q0 += chunk) {
      const int64_t m = std::min(chunk, n - q0);
      int64_t coff = 0, cbytes = 0;
      astar_dev_cells(c->H, c->W, far_cap, m, &coff, &cbytes);
      hipError_t e = hipMemcpyAsync(d_sg.p, sg4 + 4 * q0, sizeof(int32_t) * 4 * m, hipMemcpyHostToDevice, c->st);
      if (e == hipSuccess) e = hipMemsetAsync(work.p + coff, 0, (size_t)cbytes, c->st);
      if (e == hipSuccess) {
        launch_astar_dev(c->st, c->G(), d_sg.p, m, thetastar != 0, work.p, far_cap, d_path.p, cap,
                         d_len.p, d_stats.p);
        e = hipGetLastError();
      }
      if (e == hipSuccess && cap)
        e = hipMemcpyAsync(path_xy + 2 * cap * q0, d_path.p, sizeof(int64_t) * 2 * cap * m, hipMemcpyDeviceToHost, c->st);
      if (e == hipSuccess) e = hipMemcpyAsync(path_len + q0, d_len.p, sizeof(int64_t) * m, hipMemcpyDeviceToHost, c->st);
      if (e == hipSuccess) e = hipMemcpyAsync(stats4 + 4 * q0, d_stats.p, sizeof(int64_t) * 4 * m, hipMemcpyDeviceToHost, c->st);
      if (e == hipSuccess) e = hipStreamSynchronize(c->st);
      if (e != hipSuccess) rc = fail(TR_E_HIP, std::string("astar batch: ") + hipGetErrorString(e));
    }
    cleanup();
    return rc;
  })
}

int tr_steer_batch(tr_ctx* c, const double* in6, int64_t n, double* out9) {
  if (!c || n < 0 || (n && (!in6 || !out9))) return fail(TR_E_ARG, "bad steer batch");
  if (!n) return TR_OK;
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(c->fin.reserve(6 * n));
  HIPCHK(c->fout.reserve(9 * n));
  HIPCHK(hipMemcpyAsync(c->fin.p, in6, sizeof(double) * 6 * n, hipMemcpyHostToDevice, c->st));
  launch_steer(c->st, c->P, c->fin.p, n, c->fout.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out9, c->fout.p, sizeof(double) * 9 * n, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return TR_OK;
}

int tr_drive_batch(tr_ctx* c, const double* in9, int64_t n, double* out3, int32_t* ok) {
  if (!c || n < 0 || (n && (!in9 || !out3 || !ok))) return fail(TR_E_ARG, "bad drive batch");
  if (!n) return TR_OK;
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(c->fin.reserve(9 * n));
  HIPCHK(c->fout.reserve(3 * n));
  HIPCHK(c->i32.reserve(n));
  HIPCHK(hipMemcpyAsync(c->fin.p, in9, sizeof(double) * 9 * n, hipMemcpyHostToDevice, c->st));
  launch_drive(c->st, c->P, c->fin.p, n, c->fout.p, c->i32.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out3, c->fout.p, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(ok, c->i32.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return TR_OK;
}

int tr_body_clear_batch(tr_ctx* c, const double* xyt, int64_t n, double mult, uint8_t* out) {
  if (int e = need_grid(c)) return e;
  if (n < 0 || (n && (!xyt || !out))) return fail(TR_E_ARG, "bad body batch");
  if (!n) return TR_OK;
  HIPCHK(c->fin.reserve(3 * n));
  HIPCHK(c->bout.reserve(n));
  HIPCHK(hipMemsetAsync(c->err.p, 0, 4, c->st));
  HIPCHK(hipMemcpyAsync(c->fin.p, xyt, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->st));
  launch_body(c->st, c->P, c->G(), c->fin.p, n, mult, c->bout.p, c->err.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->bout.p, n, hipMemcpyDeviceToHost, c->st));
  return check_err_word(c);
}

int tr_arc_batch(tr_ctx* c, const double* in10, int64_t n, uint8_t* out) {
  if (int e = need_grid(c)) return e;
  if (n < 0 || (n && (!in10 || !out))) return fail(TR_E_ARG, "bad arc batch");
  if (!n) return TR_OK;
  HIPCHK(c->fin.reserve(10 * n));
  HIPCHK(c->bout.reserve(n));
  HIPCHK(hipMemsetAsync(c->err.p, 0, 4, c->st));
  HIPCHK(hipMemcpyAsync(c->fin.p, in10, sizeof(double) * 10 * n, hipMemcpyHostToDevice, c->st));
  launch_arc_batch(c->st, c->G(), c->fin.p, n, c->bout.p, c->err.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->bout.p, n, hipMemcpyDeviceToHost, c->st));
  return check_err_word(c);
}

static int list_common(tr_ctx* c, int64_t* out_xy, int64_t cap, int64_t* count) {
  int64_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, c->cnt.p, sizeof(int64_t), hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  *count = n;
  int64_t m = std::min(n, cap);
  if (m > 0)
    HIPCHK(hipMemcpyAsync(out_xy, c->iout.p, sizeof(int64_t) * 2 * m, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return TR_OK;
}

int tr_bresenham(tr_ctx* c, const double* seg4, int64_t* out_xy, int64_t cap, int64_t* count) {
  if (!c || !seg4 || !count || cap < 0 || (cap && !out_xy)) return fail(TR_E_ARG, "bad bresenham");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(c->fin.reserve(4));
  HIPCHK(c->cnt.reserve(1));
  HIPCHK(c->iout.reserve(2 * std::max<int64_t>(cap, 1)));
  HIPCHK(hipMemcpyAsync(c->fin.p, seg4, sizeof(double) * 4, hipMemcpyHostToDevice, c->st));
  launch_bresenham_list(c->st, c->fin.p, c->iout.p, cap, c->cnt.p);
  HIPCHK(hipGetLastError());
  return list_common(c, out_xy, cap, count);
}

int tr_circle(tr_ctx* c, double cx, double cy, double r, int64_t* out_xy, int64_t cap,
              int64_t* count) {
  if (int e = need_grid(c)) return e;
  if (!count || cap < 0 || (cap && !out_xy)) return fail(TR_E_ARG, "bad circle");
  HIPCHK(c->cnt.reserve(1));
  HIPCHK(c->iout.reserve(2 * std::max<int64_t>(cap, 1)));
  launch_circle_list(c->st, c->G(), cx, cy, r, nullptr, c->iout.p, cap, c->cnt.p);
  HIPCHK(hipGetLastError());
  return list_common(c, out_xy, cap, count);
}

int tr_arc_pixels(tr_ctx* c, const double* in10, int64_t* out_xy, int64_t cap, int64_t* count) {
  if (int e = need_grid(c)) return e;
  if (!in10 || !count || cap < 0 || (cap && !out_xy)) return fail(TR_E_ARG, "bad arc pixels");
  if (in10[9] != 0) return tr_bresenham(c, in10, out_xy, cap, count);
  HIPCHK(c->fin.reserve(10));
  HIPCHK(c->cnt.reserve(1));
  HIPCHK(c->iout.reserve(2 * std::max<int64_t>(cap, 1)));
  HIPCHK(hipMemcpyAsync(c->fin.p, in10, sizeof(double) * 10, hipMemcpyHostToDevice, c->st));
  launch_circle_list(c->st, c->G(), in10[5], in10[6], in10[7], c->fin.p, c->iout.p, cap, c->cnt.p);
  HIPCHK(hipGetLastError());
  return list_common(c, out_xy, cap, count);
}

int tr_expand_dev(tr_ctx* c, const double* d_gauss, int64_t B, const double* goal3,
                  tr_sample* d_samples, tr_record* d_records) {
  if (int e = need_grid(c)) return e;
  if (B < 0 || (B && (!d_gauss || !goal3 || !d_samples || !d_records)))
    return fail(TR_E_ARG, "bad expand");
  if (!B) return TR_OK;
  if (c->N <= 0) return fail(TR_E_STATE, "empty tree");
  return expand_batch(c, d_gauss, B, goal3, d_samples, d_records);
}

int tr_expand_dev_noalloc(tr_ctx* c, const double* d_gauss, int64_t B, const double* goal3,
                          tr_sample* d_samples, tr_record* d_records) {
  if (int e = need_grid(c)) return e;
  if (B < 0 || (B && (!d_gauss || !goal3 || !d_samples || !d_records)))
    return fail(TR_E_ARG, "bad expand");
  if (!B) return TR_OK;
  if (c->N <= 0) return fail(TR_E_STATE, "empty tree");
  if (c->st_n) return fail(TR_E_STATE, "expand_noalloc with a look-ahead staged");
  unsigned char* base = c->device < NOALLOC_MAX_DEV ? g_scratch_ptr[c->device] : nullptr;
  if (!base) return fail(TR_E_STATE, "expand_noalloc: no static scratch on this device");
  // scratch layout: query pixels, live flags, nearest nodes, the NN screen's chunk minima
  const NNPlan p = nn_plan(B, c->n_ub);
  auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
  const size_t o_qxy = 0, o_live = o_qxy + up(sizeof(int2) * (size_t)B);
  const size_t o_near = o_live + up(sizeof(int32_t) * (size_t)B);
  const size_t o_m32 = o_near + up(sizeof(int64_t) * (size_t)B);
  const size_t need = o_m32 + up(sizeof(float) * (size_t)nn_scratch(B, p));
  if (need > NOALLOC_BYTES)
    return fail(TR_E_ARG, "expand_noalloc: " + std::to_string(B) + " samples against " +
                              std::to_string(c->n_ub) + " nodes need " + std::to_string(need) +
                              " bytes of scratch, the static buffer holds " +
                              std::to_string(NOALLOC_BYTES) + " (use tr_expand_dev)");
  int2* qxy = reinterpret_cast<int2*>(base + o_qxy);
  int32_t* live = reinterpret_cast<int32_t*>(base + o_live);
  int64_t* near = reinterpret_cast<int64_t*>(base + o_near);
  float* m32 = reinterpret_cast<float*>(base + o_m32);
  launch_samples(c->st, c->P, c->G(), d_gauss, B, goal3[0], goal3[1], goal3[2], d_samples, qxy, live);
  nn_sweep(c->st, qxy, B, c->cx, c->cy, c->t4.p, c->d_count.p, p, m32);
  nn_resolve(c->st, qxy, B, c->cx, c->cy, c->txy.p, c->d_count.p, p, c->d_maxabs.p, sample_qmax(c),
             m32, near, nullptr);
  launch_expand_arc(c->st, c->P, c->G(), near, B, d_samples, live, c->txy.p, c->tth.p, goal3[0],
                    goal3[1], goal3[2], c->htab.p, c->hmask, c->dd_err.p, d_records);
  HIPCHK(hipGetLastError());
  return TR_OK;
}

int tr_rng_set_state(tr_ctx* c, const uint32_t* key624, int32_t pos, int32_t has_gauss,
                     double gauss) {
  if (!c || !key624 || pos < 0 || pos > 624) return fail(TR_E_ARG, "bad MT19937 state");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    HIPCHK(hipStreamSynchronize(c->st));
    HIPCHK(hipStreamSynchronize(c->rng_st));
    if (c->rng_rs < 3 * 624) {
      c->rng_ring.release();
      HIPCHK(c->rng_ring.reserve(3 * 624));
      c->rng_rs = 3 * 624;
    }
    HIPCHK(copy_sync(c->st, c->rng_ring.p, key624, 624 * sizeof(uint32_t), hipMemcpyHostToDevice));
    const int64_t ge[2] = {624, 0};
    const RngPos p{pos, has_gauss ? 1 : 0, 0, has_gauss ? gauss : 0.0};
    HIPCHK(copy_sync(c->st, c->rng_gen.p, ge, sizeof(ge), hipMemcpyHostToDevice));
    HIPCHK(copy_sync(c->st, c->rng_pos.p, &p, sizeof(p), hipMemcpyHostToDevice));
    HIPCHK(fill_sync(c->st, c->rng_err.p, 0, sizeof(int32_t)));
    c->rng_on = true;
    return TR_OK;
  })
}

int tr_rng_get_state(tr_ctx* c, uint32_t* key624, int32_t* pos, int32_t* has_gauss, double* gauss) {
  if (!c || !key624 || !pos || !has_gauss || !gauss) return fail(TR_E_ARG, "NULL argument");
  if (!c->rng_on) return fail(TR_E_STATE, "no gaussian stream: call tr_rng_set_state");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(hipStreamSynchronize(c->st));
  HIPCHK(hipStreamSynchronize(c->rng_st));
  if (int e = rng_check(c)) return e;
  RngPos p;
  HIPCHK(copy_sync(c->st, &p, c->rng_pos.p, sizeof(p), hipMemcpyDeviceToHost));
  // numpy's (key, 624) and (next key, 0) name the same stream position: report the former
  const int64_t blk = p.wpos > 0 && p.wpos % 624 == 0 ? p.wpos / 624 - 1 : p.wpos / 624;
  HIPCHK(copy_sync(c->st, key624, c->rng_ring.p + (624 * blk) % c->rng_rs, 624 * sizeof(uint32_t),
                   hipMemcpyDeviceToHost));
  *pos = (int32_t)(p.wpos - 624 * blk);
  *has_gauss = p.has;
  *gauss = p.has ? p.gauss : 0.0;
  return TR_OK;
}

int tr_rng_gauss_dev(tr_ctx* c, int64_t n, double* d_out) {
  if (!c || n < 0 || (n && !d_out)) return fail(TR_E_ARG, "bad gaussian draw");
  if (!n) return TR_OK;
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    if (int e = rng_ensure(c, n)) return e;
    HIPCHK(hipStreamSynchronize(c->rng_st));
    RngPos* scratch = c->rng_pos.p + 1 + 8 * tr_ctx::RC;
    rng_chunk(c->st, c->rng_ring.p, c->rng_rs, c->rng_gen.p, c->rng_pos.p, n, n, d_out, scratch,
              c->rng_cnt.p, c->rng_err.p, c->rng_seeds.p, c->rng_done.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->rng_pos.p, scratch, sizeof(RngPos), hipMemcpyDeviceToDevice, c->st));
    return TR_OK;
  })
}

int tr_enable_timing(tr_ctx* c, int level) {
  if (!c) return fail(TR_E_ARG, "ctx is NULL");
  c->timing = level < 0 ? 0 : (level > 2 ? 1 : level);
  c->tmask = level == 3 ? 0u : 3u;                 // 3: level 1's events on every batch
  return TR_OK;
}

int tr_last_timings(const tr_ctx* c, double* us5) {
  if (!c || !us5) return fail(TR_E_ARG, "NULL argument");
  if (!c->timing) return fail(TR_E_STATE, "timing disabled");
  memcpy(us5, c->t_us, sizeof(c->t_us));
  return TR_OK;
}

int tr_last_nn_timings(const tr_ctx* c, double* us3) {
  if (!c || !us3) return fail(TR_E_ARG, "NULL argument");
  if (!c->timing) return fail(TR_E_STATE, "timing disabled");
  memcpy(us3, c->nn_us, sizeof(c->nn_us));
  return TR_OK;
}

int tr_last_host_timings(const tr_ctx* c, double* us3) {
  if (!c || !us3) return fail(TR_E_ARG, "NULL argument");
  memcpy(us3, c->host_us, sizeof(c->host_us));
  return TR_OK;
}

// ------------------------------------------------------------------ book
int tr_book_create(tr_book** out) {
  if (!out) return fail(TR_E_ARG, "out is NULL");
  GUARD({
    *out = new tr_book();
    return TR_OK;
  })
}
int tr_book_destroy(tr_book* b) {
  delete b;
  return TR_OK;
}
int tr_book_reset(tr_book* b, const double* s) {
  if (!b || !s) return fail(TR_E_ARG, "NULL argument");
  GUARD({
    b->reset(s);
    return TR_OK;
  })
}
int tr_book_set_straight_reject(tr_book* b, int on) {
  if (!b) return fail(TR_E_ARG, "book is NULL");
  b->straight_reject = on != 0;
  return TR_OK;
}
int tr_book_ingest(tr_book* b, const tr_sample* s, const tr_record* r, int64_t n, int64_t n_snap,
                   int64_t* n_new, int64_t* sol) {
  if (!b || n < 0 || (n && (!s || !r)) || !n_new || !sol) return fail(TR_E_ARG, "bad ingest");
  GUARD({ return b->ingest(s, r, n, n_snap, n_new, sol); })
}
int tr_book_reserve(tr_book* b, int64_t nodes, int64_t edges) {
  if (!b || nodes < 0 || edges < 0) return fail(TR_E_ARG, "bad book reserve");
  GUARD({
    reserve_touched(b->xyt, 3 * (size_t)nodes);
    reserve_touched(b->parent, (size_t)nodes);
    reserve_touched(b->u6, 6 * (size_t)nodes);
    reserve_touched(b->e_par, (size_t)edges);
    reserve_touched(b->e_child, (size_t)edges);
    return TR_OK;
  })
}

int tr_book_replay(tr_book* b, const tr_resolved* rs, int64_t n, int64_t* n_new, int64_t* sol) {
  if (!b || n < 0 || (n && !rs) || !n_new || !sol) return fail(TR_E_ARG, "bad replay");
  GUARD({ return b->replay(rs, n, n_new, sol); })
}
int64_t tr_book_size(const tr_book* b) { return b ? b->size() : -1; }
int64_t tr_book_edges(const tr_book* b) { return b ? (int64_t)b->e_par.size() : -1; }
int tr_book_nodes(const tr_book* b, int64_t from, int64_t to, double* xyt) {
  if (!b || from < 0 || to > b->size() || from > to || (to > from && !xyt))
    return fail(TR_E_ARG, "bad node range");
  memcpy(xyt, b->xyt.data() + 3 * from, sizeof(double) * 3 * (size_t)(to - from));
  return TR_OK;
}
int tr_book_export(const tr_book* b, int64_t* parent, double* u6, int64_t* e_off, int64_t* e_child) {
  if (!b) return fail(TR_E_ARG, "book is NULL");
  const int64_t n = b->size(), m = (int64_t)b->e_par.size();
  if (parent) memcpy(parent, b->parent.data(), sizeof(int64_t) * (size_t)n);
  if (u6) memcpy(u6, b->u6.data(), sizeof(double) * 6 * (size_t)n);
  if (e_off && e_child) {  // stable counting sort of edges by parent = per-node append order
    std::vector<int64_t> cnt((size_t)n + 1, 0);
    for (int64_t k = 0; k < m; ++k) cnt[(size_t)b->e_par[k] + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
    memcpy(e_off, cnt.data(), sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t k = 0; k < m; ++k) e_child[cnt[(size_t)b->e_par[k]]++] = b->e_child[k];
  }
  return TR_OK;
}

// ------------------------------------------------------------------ RRT session
int tr_rrt_begin(tr_ctx* c, const double* start3, const double* goal3) {
  if (int e = need_grid(c)) return e;
  if (!start3 || !goal3) return fail(TR_E_ARG, "NULL argument");
  GUARD({
    worker_drain(c);                         // batches of an earlier session are abandoned
    worker_start(c);
    c->r_head = c->r_tail = c->r_count = 0;
    c->w_next = 0;
    c->book_err = 0;
    c->book_msg.clear();
    c->book_sol = -1;
    c->w_dev_nodes = 1;
    c->book.reset(start3);
    if (int e = tr_tree_reset(c, std::max<int64_t>(c->txy.cap, 1024))) return e;
    if (int e = tr_tree_append(c, start3, 1)) return e;
    HIPCHK(hipEventRecord(c->ev_dd, c->st));
    c->ev_latest = c->ev_dd;
    HIPCHK(c->dd_done.reserve(1));
    const unsigned long long ep = c->epoch;          // no dedupe yet in this session: done
    HIPCHK(copy_sync(c->st, c->dd_done.p, &ep, sizeof(ep), hipMemcpyHostToDevice));
    c->next_k = 0;
    c->st_n = 0;
    memcpy(c->goal, goal3, sizeof(c->goal));
    c->session = true;
    return TR_OK;
  })
}

tr_book* tr_rrt_book(tr_ctx* c) { return c ? &c->book : nullptr; }

int tr_rrt_reserve(tr_ctx* c, int64_t nodes, int64_t batch) {
  if (!c || nodes < 0 || batch < 0) return fail(TR_E_ARG, "bad reserve");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    if (int e = ensure_tree(c, nodes)) return e;
    if (int e = ensure_table(c, nodes)) return e;
    if (int e = ensure_dd_scratch(c, batch)) return e;
    for (int k = 0; k < tr_ctx::R; ++k)
      if (int e = ensure_slot(c, k, batch)) return e;
    // the per-batch scratch sets of this rank's slice (a set that has to grow mid-run drains
    // both streams first: measured ~0.8 ms per step at 32768 samples while the tree, and with it
    // the NN screen's chunk count, kept outgrowing the sets)
    const int64_t b = (batch + c->world - 1) / std::max(c->world, 1);
    if (b > 0) {
      for (int k = 0; k < tr_ctx::NS; ++k) {
        if (int e = grow(c, c->s_qxy[k], b)) return e;
        if (int e = grow(c, c->s_live[k], b)) return e;
        if (int e = grow(c, c->s_near[k], b)) return e;
        if (int e = grow(c, c->s_dnear[k], b)) return e;
        // (the sweep's scratch: whole batches while the tree is sparse, the far list after)
        if (int e = grow(c, c->s_m32[k], nn_scratch_ub(b, std::max<int64_t>(nodes, 1)))) return e;
      }
      if (int e = grow(c, c->chg, b)) return e;
      if (cells_possible(c)) {                    // both streams' cell sets, sized for the reserved tree
        if (int e = cells_alloc(c, 0)) return e;
        if (int e = cells_alloc(c, 1)) return e;
      }
    }
    reserve_touched(c->book.xyt, 3 * (size_t)nodes);
    reserve_touched(c->book.parent, (size_t)nodes);
    reserve_touched(c->book.u6, 6 * (size_t)nodes);
    reserve_touched(c->book.e_par, (size_t)nodes + 4 * (size_t)batch);
    reserve_touched(c->book.e_child, (size_t)nodes + 4 * (size_t)batch);
    return TR_OK;
  })
}

int tr_rrt_pipe_expand(tr_ctx* c, const double* d_gauss, int64_t B, tr_sample* d_samples,
                       tr_record* d_records) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (B <= 0 || !d_gauss || !d_samples || !d_records) return fail(TR_E_ARG, "bad pipe_expand");
  if (set_dev(c)) return TR_E_HIP;
  return expand_batch(c, d_gauss, B, c->goal, d_samples, d_records);
}

int tr_rrt_pipe_stage(tr_ctx* c, const double* d_gauss, int64_t B, tr_sample* d_samples,
                      tr_record* d_records) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (B <= 0 || !d_gauss || !d_samples || !d_records) return fail(TR_E_ARG, "bad pipe_stage");
  if (c->st_n == tr_ctx::SQ) return fail(TR_E_STATE, "pipe_stage: two staged batches are pending");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({ return stage_batch(c, d_gauss, B, d_samples, d_records); })
}

int tr_rrt_pipe_dedupe(tr_ctx* c, const tr_sample* d_samples, const tr_record* d_records, int64_t n) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (n < 0 || (n && !d_records)) return fail(TR_E_ARG, "bad pipe_dedupe");
  (void)d_samples;                             // membership is in the records (TR_FL_MEMBER)
  if (c->r_count == tr_ctx::R) return fail(TR_E_STATE, "commit ring full: call tr_rrt_pipe_commit");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    const int k = c->r_head;
    if (int e = ensure_tree(c, c->n_ub + n)) return e;
    if (int e = ensure_table(c, c->n_ub + n)) return e;
    if (int e = ensure_dd_scratch(c, n)) return e;
    if (int e = ensure_slot(c, k, n)) return e;
    if (int e = ensure_bins(c, n)) return e;
    c->epoch++;
    c->db_ok[c->epoch & 3] = 0;
    if (c->timing > 1) HIPCHK(hipEventRecord(c->t_ev[4], c->st));
    const int ms = c->tm_pending;
    if (ms >= 0) HIPCHK(hipEventRecord(c->tm_ev[ms][3], c->st));
    if (n) {
      DDArgs a;
      a.rec = d_records;
      a.n = n;
      a.txy = c->txy.p;
      a.t4 = c->t4.p;
      a.tth = c->tth.p;
      a.count = c->d_count.p;
      a.snap = c->snap.p + (c->epoch & 3);
      a.htab = c->htab.p;
      a.hmask = c->hmask;
      a.maxabs = c->d_maxabs.p;
      a.cx = c->cx;
      a.cy = c->cy;
      a.err = c->dd_err.p;
      a.claim = dd_claim_args(c);
      a.slot = c->dd_slot.p;
      a.lr = c->dd_lr.p;
      a.bc = c->dd_bc.p;
      a.base = c->dd_base.p;
      a.out = c->commit_view(k);
      a.done = c->gate ? c->dd_done.p : nullptr;
      a.blocks = c->dd_blocks.p;
      a.ready = c->gate ? c->r_ready.p + k : nullptr;
      a.ticket = c->dd_ticket.p;
      a.bst = c->dd_bst.p;
      a.idxs = c->dd_idx.p;
      a.gate = nullptr;
      a.gate_v = 0;
      // the next staged batch's gate rides at the end of this k_dd (one launch less on the
      // batch's stream); its look-ahead is already enqueued on the side stream
      // one kernel for batches of up to dd_fused_max records (its blocks wait for every earlier
      // block: past a few dozen blocks the polling costs more than two more launches; cfg3's
      // 65536 records: 1.8 ms fused vs 0.42 ms in three kernels, profiles/r02/cfg3/)
      const bool fused = c->dd_fused && n <= c->dd_fused_max;
      if (c->gate && fused && c->dd_gatefold && c->st_n > 0) {
        a.gate = c->st_done.p;
        a.gate_v = c->stq[0].seq;
        c->gated_seq = c->stq[0].seq;
      }
      if (fused) {
        a.claim.blast = nullptr;
        a.done = c->dd_done.p;                         // k_dd publishes every epoch
      }
      if (c->delta_bins && c->db_cnt.p) {              // the new nodes by bin, for the correction
        const int set = (int)(c->epoch & 3);
        const int64_t nb = (int64_t)c->db_nbx * c->db_nby + 1;
        if (c->db_zero[set] != c->epoch)               // (the dedupe before this one filed nothing)
          HIPCHK(hipMemsetAsync(c->db_cnt.p + set * nb, 0, sizeof(uint32_t) * nb, c->st));
        a.bins = c->bins_view();
        c->db_ok[set] = c->epoch;
        c->db_zero[(set + 1) & 3] = c->epoch + 1;
      }
      dd_batch(c->st, a, fused);
    } else {
      HIPCHK(hipMemcpyAsync(c->snap.p + (c->epoch & 3), c->d_count.p, sizeof(int64_t),
                            hipMemcpyDeviceToDevice, c->st));
      DHead z{};
      z.pad = head_tag(c->epoch);
      memcpy(c->commit_view(k).head, &z, sizeof(z));   // (slot idle: no batch in flight uses it)
      if (c->gate) {                                     // no kernel publishes this epoch
        launch_publish(c->st, c->dd_done.p, c->epoch);
        launch_publish(c->st, c->r_ready.p + k, c->epoch);
      }
    }
    if (c->timing > 1) HIPCHK(hipEventRecord(c->t_ev[5], c->st));
    if (ms >= 0) {
      HIPCHK(hipEventRecord(c->tm_ev[ms][4], c->st));
      c->tm_used[ms] = true;
      c->tm_pending = -1;
    }
    HIPCHK(hipGetLastError());
    if (!c->gate) {                          // device-side edge first, then the host's event
      HIPCHK(hipEventRecord(c->ev_dd, c->st));
      c->ev_latest = c->ev_dd;
    }
    c->r_epoch[k] = c->epoch;
    c->r_stream[k] = c->st;
    if (!c->gate) HIPCHK(hipEventRecord(c->r_ev[k], c->st));   // gate mode: r_ready[k]

    c->r_n[k] = n;
    c->r_head = (k + 1) % tr_ctx::R;
    c->r_count++;
    c->n_ub += n;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->r_done[k] = false;
      c->w_pending++;
    }
    c->cv_work.notify_one();
    return TR_OK;
  })
}

int tr_rrt_pipe_commit(tr_ctx* c, int64_t* n_nodes, int64_t* sol) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session");
  if (!n_nodes || !sol) return fail(TR_E_ARG, "bad pipe_commit");
  if (!c->r_count) return fail(TR_E_STATE, "pipe_commit: nothing in flight");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    const int k = c->r_tail;
    const double t0 = now_us();
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv_done.wait(lk, [c, k] { return c->r_done[k]; });
    }
    const double t1 = now_us();
    if (c->timing && c->r_count == 1) {   // the batch just waited for is the last timed one
      float a = 0, b = 0, d = 0, e = 0;
      // level 1 times the nearest-node work where it runs: the side stream's sweep of a staged
      // batch, else the main stream's sweep + resolve (each event costs GPU idle time)
      if (c->timing > 1 || !c->last_staged) HIPCHK(hipEventElapsedTime(&a, c->t_ev[0], c->t_ev[1]));
      if (c->timing > 1) {
        HIPCHK(hipEventElapsedTime(&b, c->t_ev[1], c->t_ev[2]));
        HIPCHK(hipEventElapsedTime(&d, c->t_ev[2], c->t_ev[3]));
        HIPCHK(hipEventElapsedTime(&e, c->t_ev[4], c->t_ev[5]));
      }
      c->t_us[0] = a * 1e3; c->t_us[1] = b * 1e3; c->t_us[2] = d * 1e3; c->t_us[3] = e * 1e3;
      c->t_us[4] = (a + b + d + e) * 1e3;
      c->nn_us[1] = a * 1e3;
      float sd = 0;
      if (c->ts_last >= 0 && c->ts_used[c->ts_last] &&
          hipEventQuery(c->ts_ev[c->ts_last][2]) == hipSuccess &&
          hipEventElapsedTime(&sd, c->ts_ev[c->ts_last][0], c->ts_ev[c->ts_last][2]) == hipSuccess)
        c->nn_us[0] = sd * 1e3;
      (void)hipGetLastError();          // a failed query must not surface in a later check
    }
    const int rc = c->r_rc[k];
    const int64_t n = c->r_n[k], dev_new = c->r_devnew[k];
    *sol = c->r_sol[k];
    c->r_tail = (k + 1) % tr_ctx::R;
    c->r_count--;
    c->N = c->r_nodes[k];
    c->n_ub -= n - dev_new;
    *n_nodes = c->N;
    c->host_us[0] = t1 - t0;
    c->host_us[1] = c->r_rep_us[k];
    c->host_us[2] = 0;
    if (rc) return fail(rc, c->r_msg[k]);
    return TR_OK;
  })
}

int tr_rrt_pending(const tr_ctx* c) { return c ? c->r_count : -1; }

int tr_comm_unique_id(uint8_t* id128) {
  if (!id128) return fail(TR_E_ARG, "NULL argument");
  const Rccl* r = rccl();
  if (!r) return fail(TR_E_STATE, "librccl.so.1 not found");
  ncclUniqueId id;
  const ncclResult_t e = r->get_id(&id);
  if (e != ncclSuccess) return fail(TR_E_HIP, std::string("ncclGetUniqueId: ") + r->err(e));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  memcpy(id128, &id, 128);
  return TR_OK;
}

int tr_comm_init_host(tr_ctx* c, int rank, int world, tr_host_gather_fn fn, void* user) {
  if (!c || !fn || world < 1 || rank < 0 || rank >= world) return fail(TR_E_ARG, "bad comm init");
  if (c->sharded()) return fail(TR_E_STATE, "communicator already initialised");
  c->hg_fn = fn;
  c->hg_user = user;
  c->rank = rank;
  c->world = world;
  return TR_OK;
}

int tr_comm_init(tr_ctx* c, int rank, int world, const uint8_t* id128) {
  if (!c || !id128 || world < 1 || rank < 0 || rank >= world) return fail(TR_E_ARG, "bad comm init");
  if (c->sharded()) return fail(TR_E_STATE, "communicator already initialised");
  if (set_dev(c)) return TR_E_HIP;
  const Rccl* r = rccl();
  if (!r) return fail(TR_E_STATE, "librccl.so.1 not found");
  ncclUniqueId id;
  memcpy(&id, id128, 128);
  const ncclResult_t e = r->init(&c->comm, world, id, rank);
  if (e != ncclSuccess) {
    c->comm = nullptr;
    return fail(TR_E_HIP, std::string("ncclCommInitRank: ") + r->err(e));
  }
  c->rank = rank;
  c->world = world;
  return TR_OK;
}

// Rank-order all-gather of `bytes` per rank on the context stream: RCCL, or the host hook (sync,
// D2H of this rank's bytes, fn, H2D of every rank's).
static int comm_all_gather(tr_ctx* c, const void* d_send, void* d_recv, int64_t bytes) {
  if (c->comm) {
    const Rccl* r = rccl();
    const ncclResult_t e = r->all_gather(d_send, d_recv, (size_t)bytes, ncclUint8, c->comm, c->st);
    if (e != ncclSuccess) return fail(TR_E_HIP, std::string("ncclAllGather: ") + r->err(e));
    return TR_OK;
  }
  HIPCHK(c->hg_send.reserve(bytes));
  HIPCHK(c->hg_recv.reserve(bytes * c->world));
  HIPCHK(hipMemcpyAsync(c->hg_send.p, d_send, (size_t)bytes, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  if (int e = c->hg_fn(c->hg_user, c->hg_send.p, c->hg_recv.p, bytes))
    return fail(TR_E_STATE, "host gather hook failed (" + std::to_string(e) + ")");
  HIPCHK(hipMemcpyAsync(d_recv, c->hg_recv.p, (size_t)(bytes * c->world), hipMemcpyHostToDevice, c->st));
  HIPCHK(hipStreamSynchronize(c->st));   // the pinned buffers are reused by the next gather
  return TR_OK;
}

int tr_rrt_run(tr_ctx* c, const double* d_gauss, int64_t B, int64_t rows, tr_sample* d_samples,
               tr_record* d_records, tr_sample* d_samples_all, tr_record* d_records_all, int lag,
               int stage, int64_t* n_nodes, int64_t* sol) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (B <= 0 || rows < 0 || !n_nodes || !sol || (!d_samples != !d_records))
    return fail(TR_E_ARG, "bad rrt_run");
  const bool own_rng = d_gauss == nullptr;   // the engine draws the gaussians itself (rng.hip)
  if (own_rng && !c->rng_on) return fail(TR_E_STATE, "rrt_run without gaussians: call tr_rng_set_state");
  const bool shard = c->sharded();
  const int64_t W = shard ? c->world : 1, BT = B * W;
  if (lag < 1 || lag >= tr_ctx::R) return fail(TR_E_ARG, "rrt_run: lag must be in [1, 5]");
  if (c->r_count) return fail(TR_E_STATE, "rrt_run with pipelined batches in flight");
  if (set_dev(c)) return TR_E_HIP;
  GUARD({
    for (int q = 0; q < 5; ++q) c->run_us[q] = 0;
    for (int q = 0; q < 3; ++q) c->run_nn[q] = c->run_host[q] = 0;
    c->run_n = 0;
    if (c->timing) {                   // the sums cover this run's sampled batches only
      harvest_all_side(c);
      harvest_all_main(c);
      c->ts_sum[0] = c->ts_sum[1] = 0;
      c->ts_n = 0;
      c->tm_sum[0] = c->tm_sum[1] = c->tm_sum[2] = 0;
      c->tm_n = 0;
      c->tm_pending = -1;
    }
    *sol = -1;
    *n_nodes = c->N;
    int rc = TR_OK;
    double t_run[4] = {c->trace_on ? now_us() : 0.0, 0, 0, 0};   // entry, loop end, committed, rng synced
    c->stage_n = 0;
    c->trace_t0 = t_run[0];
    int64_t n_commit = 0, goal_batch = -1, fail_batch = -1;   // batches of this run, in order
    auto commit = [&]() {
      int64_t nn = 0, sl = -1;
      const int e = tr_rrt_pipe_commit(c, &nn, &sl);
      const int64_t b = n_commit++;
      *n_nodes = nn;
      if (sl >= 0 && *sol < 0) { *sol = sl; goal_batch = b; }
      if (e && fail_batch < 0) fail_batch = b;
      for (int q = 0; q < 3; ++q) c->run_host[q] += c->host_us[q];
      c->run_n++;
      return e;
    };
    // look-ahead depth (0 off); the caller's sample / record buffers hold nslot sets of B
    const int depth = std::min(std::max(stage, 0), tr_ctx::SQ);
    const int nslot = std::max(2, depth + 1);
    if (!d_samples) {                  // engine-owned sets
      if (int e = grow(c, c->samp, nslot * B)) return e;
      if (int e = grow(c, c->rec, nslot * B)) return e;
      d_samples = c->samp.p;
      d_records = c->rec.p;
    }
    if (shard && !d_records_all) {
      if (int e = grow(c, c->rec_all, 2 * BT)) return e;
      d_records_all = c->rec_all.p;
    }
    // Engine-drawn gaussians: chunk q = batches [q C, (q + 1) C) in slot q & 1, drawn on the rng
    // stream once the slot's previous chunk (q - 2) is consumed; chunk i / C + 1 is enqueued at
    // batch i (i % C == 0), so with C >= the look-ahead depth every batch's chunk is enqueued
    // before its sample kernel.  Every rank draws the whole BT stream and reads its slice.
    const int64_t G3 = 3 * BT;
    const int64_t C = own_rng ? std::max<int64_t>(std::max(2, depth),
                                                  std::min<int64_t>(tr_ctx::RC, 49152 / G3))
                              : 1;
    if (own_rng) {
      if (int e = rng_ensure(c, C * G3)) return e;
      if (int e = grow(c, c->rng_out, 2 * C * G3)) return e;
      HIPCHK(hipStreamSynchronize(c->rng_st));
      // a tr_rng_gauss_dev still in flight on the context stream owns the stream position, the
      // ring and the count scratch: the run's chunks (rng stream) start after it
      HIPCHK(hipEventRecord(c->rng_free, c->st));
      HIPCHK(hipStreamWaitEvent(c->rng_st, c->rng_free, 0));
    }
    // The run's first chunk is enqueued batch by batch, each batch only when the loop first needs
    // it (c0_upto): a run's first expansion is then enqueued after one batch's launches, not after
    // the chunk's (16 launches at four batches: ~80 us of host time before the first kernel of
    // the run's first batch).  c0_next = batches of chunk 0 enqueued so far.
    const int64_t c0_nb = own_rng && std::min(C, rows) > 1 ? std::min(C, rows) : 0;
    int64_t c0_next = 0;
    auto c0_upto = [&](int64_t j) -> int {
      j = std::min(j, c0_nb - 1);
      RngPos* bstate = c->rng_pos.p + 1;
      for (; c0_next <= j; ++c0_next) {
        const int64_t b = c0_next;
        rng_chunk(c->rng_st, c->rng_ring.p, c->rng_rs, c->rng_gen.p, b ? bstate + b - 1 : c->rng_pos.p,
                  G3, G3, c->rng_out.p + b * G3, bstate + b, c->rng_cnt.p, c->rng_err.p,
                  c->rng_seeds.p, c->rng_done.p);
        if (b == 0 && c->gate) launch_publish(c->rng_st, c->rng_flag.p, ++c->rng_seq);
        HIPCHK(hipEventRecord(c->rng_b[b], c->rng_st));
        if (b == c0_nb - 1) {              // the chunk's end: its event and the kept key blocks
          HIPCHK(hipEventRecord(c->rng_ev[0], c->rng_st));
          rng_keep(c->rng_st, c->rng_ring.p, c->rng_rs, bstate, c0_nb, c->rng_keys.p);
        }
      }
      HIPCHK(hipGetLastError());
      return TR_OK;
    };
    auto enqueue_chunk = [&](int64_t q) -> int {
      const int64_t nb = std::min(C, rows - q * C);
      if (nb <= 0) return TR_OK;
      if (q == 0 && nb > 1) return c0_upto(0);
      if (q == 1 && c0_next < c0_nb)       // (chunk 0 is drawn first: the stream's order)
        if (int e = c0_upto(c0_nb - 1)) return e;
      const int sl = (int)(q & 1);
      if (q >= 2) {                      // batches < q C - C (chunk q - 2) are all expanded
        HIPCHK(hipEventRecord(c->rng_free, c->st));
        HIPCHK(hipStreamWaitEvent(c->rng_st, c->rng_free, 0));
      }
      const RngPos* start = q == 0 ? c->rng_pos.p : c->rng_pos.p + 1 + ((q - 1) & 7) * tr_ctx::RC + (C - 1);
      RngPos* bstate = c->rng_pos.p + 1 + (q & 7) * tr_ctx::RC;
      double* out = c->rng_out.p + sl * C * G3;
      // (the run's first chunk of more than one batch goes batch by batch, each with its own
      // event, through c0_upto: the first batch and the first look-aheads wait for one batch's
      // words each, not the chunk's; the generator is one serial workgroup, 23 us per batch)
      rng_chunk(c->rng_st, c->rng_ring.p, c->rng_rs, c->rng_gen.p, start, nb * G3, G3, out, bstate,
                c->rng_cnt.p, c->rng_err.p, c->rng_seeds.p, c->rng_done.p);
      HIPCHK(hipEventRecord(c->rng_ev[sl], c->rng_st));
      rng_keep(c->rng_st, c->rng_ring.p, c->rng_rs, c->rng_pos.p + 1 + (q & 7) * tr_ctx::RC, nb,
               c->rng_keys.p + (q & 7) * tr_ctx::RC * 624);
      HIPCHK(hipGetLastError());
      return TR_OK;
    };
    auto row = [&](int64_t j) -> const double* {          // rank's slice of batch j's gaussians
      if (own_rng) return c->rng_out.p + ((j / C) & 1) * C * G3 + (j % C) * G3 + 3 * B * c->rank;
      return d_gauss + G3 * j + 3 * B * c->rank;
    };
    int64_t rng_waited[2] = {INT64_MIN, INT64_MIN};   // per stream (main, side): the chunk last waited for
    const bool first_apart = own_rng && std::min(C, rows) > 1;   // chunk 0: an event per batch
    auto rng_wait = [&](hipStream_t s, int64_t j) -> int {
      // a stream waits for a chunk's event once (stream order covers its later batches); each
      // hipStreamWaitEvent costs host time on the enqueue path
      int64_t& last = rng_waited[s == c->side ? 1 : 0];
      const int64_t id = first_apart && j < C ? -1 - j : j / C;
      if (own_rng && last != id) {
        if (c->gate && id == -1 && s == c->st)
          launch_gate(s, c->rng_flag.p, c->rng_seq, c->dd_err.p);
        else
          HIPCHK(hipStreamWaitEvent(s, id < 0 ? c->rng_b[j] : c->rng_ev[(j / C) & 1], 0));
        last = id;
      }
      return TR_OK;
    };
    if (own_rng && rows > 0 && (rc = enqueue_chunk(0))) return rc;
    bool chunk1_due = false;             // chunk 1 waits for the first batch's launches
    auto rng_need = [&](int64_t j) -> int {   // batch j's gaussians are enqueued on the rng stream
      if (!own_rng) return TR_OK;
      if (j < C) return c0_upto(j);
      if (chunk1_due) {
        chunk1_due = false;
        return enqueue_chunk(1);
      }
      return TR_OK;
    };
    int64_t staged_to = 0;               // batches [.., staged_to) have been staged
    int64_t i = 0;
    for (; i < rows && *sol < 0 && !rc; ++i) {
      const int k = (int)(i % nslot);
      if (own_rng && i % C == 0) {
        // (the run's first batch: its own launches first, the rest of chunk 0 and chunk 1 after)
        if (i == 0) chunk1_due = true;
        else if ((rc = enqueue_chunk(i / C + 1))) break;
      }
      const double* g = row(i);
      tr_sample* smp = d_samples + k * B;
      tr_record* rec = d_records + k * B;
      const double te = now_us();       // host time spent enqueueing this batch (run_host[2])
      double* tr = c->trc[c->enq_seq++ % tr_ctx::TRN];
      if (c->trace_on) tr[0] = te;
      if ((rc = rng_need(i)) || (rc = rng_wait(c->st, i))) break;
      if ((rc = tr_rrt_pipe_expand(c, g, B, smp, rec))) break;
      if (c->trace_on) tr[1] = now_us();
      for (int64_t j = std::max(staged_to, i + 1); j <= i + depth && j < rows && !rc; ++j) {
        const int kj = (int)(j % nslot);
        if ((rc = rng_need(j)) || (rc = rng_wait(c->side, j))) break;
        rc = stage_batch(c, row(j), B, d_samples + kj * B, d_records + kj * B);
        staged_to = j + 1;
      }
      if (rc) break;
      if (c->trace_on) tr[2] = now_us();
      if (shard) {                     // rank order = global sample order
        tr_sample* sa = d_samples_all + (i & 1) * BT;
        tr_record* ra = d_records_all + (i & 1) * BT;
        (void)sa;                      // the records carry the snapshot lookups: one all-gather
        if ((rc = comm_all_gather(c, rec, ra, sizeof(tr_record) * B))) break;
        if ((rc = tr_rrt_pipe_dedupe(c, nullptr, ra, BT))) break;
      } else {
        if ((rc = tr_rrt_pipe_dedupe(c, smp, rec, B))) break;
      }
      c->run_host[2] += now_us() - te;
      if (c->trace_on) tr[3] = now_us();
      if (chunk1_due) {
        chunk1_due = false;
        if ((rc = enqueue_chunk(1))) break;
      }
      while (c->r_count > lag && !rc) {
        rc = commit();
        if (c->trace_on) c->trc[c->com_seq++ % tr_ctx::TRN][4] = now_us();
      }
    }
    if (c->trace_on) t_run[1] = now_us();
    if (own_rng) {                       // (a run that stopped inside its first chunk: the chunk's kept keys)
      const int e = c0_upto(c0_nb - 1);
      if (!rc) rc = e;
    }
    // The stream ends after the last batch the run used (the ring has moved on past it when the
    // run looked ahead: re-seed from its kept block).  With every batch enqueued and no goal so
    // far that is most likely the last one: rebased now, beside the batches still in flight, and
    // again below should a goal or an error turn up in them.
    auto rebase_to = [&](int64_t L) -> int {
      const int64_t at = ((L / C) & 7) * tr_ctx::RC + L % C;
      rng_rebase(c->rng_st, c->rng_ring.p, c->rng_gen.p, c->rng_pos.p, c->rng_pos.p + 1 + at,
                 c->rng_keys.p + at * 624);
      HIPCHK(hipGetLastError());
      // the stream's error word rides the same synchronization (every chunk ran on this stream)
      HIPCHK(hipMemcpyAsync(c->rng_err_h.p, c->rng_err.p, sizeof(int32_t), hipMemcpyDeviceToHost, c->rng_st));
      return TR_OK;
    };
    const bool early = own_rng && !rc && *sol < 0 && i == rows && rows > 0;
    if (early && (rc = rebase_to(rows - 1))) return rc;
    if (c->st_n) {                       // look-aheads past the goal / an error: drop them
      HIPCHK(hipStreamSynchronize(c->side));
      c->st_n = 0;
    }
    while (c->r_count) {
      const int e = commit();
      if (!rc) rc = e;
    }
    if (c->trace_on) t_run[2] = now_us();
    if (own_rng && n_commit > 0) {
      const int64_t L = goal_batch >= 0 ? goal_batch : (fail_batch >= 0 ? fail_batch : n_commit - 1);
      if (!(early && L == rows - 1))
        if (int e = rebase_to(L)) return e;
      HIPCHK(hipStreamSynchronize(c->rng_st));
      if (c->rng_err_h.p[0]) return rng_check(c);
    }
    if (c->trace_on) {
      t_run[3] = now_us();
      fprintf(stderr, "run of %lld batches, us since entry: loop done %.1f, committed %.1f, rng stream "
              "rebased %.1f; first batch enqueued at %.1f\n", (long long)rows, t_run[1] - t_run[0],
              t_run[2] - t_run[0], t_run[3] - t_run[0],
              c->trc[(c->enq_seq - std::min<int64_t>(c->enq_seq, i)) % tr_ctx::TRN][0] - t_run[0]);
      fprintf(stderr, "stage calls us (sum): wait %.1f samples %.1f sweep %.1f resolve %.1f record %.1f\n",
              c->stage_us[0], c->stage_us[1], c->stage_us[2], c->stage_us[3], c->stage_us[4]);
      for (double& v : c->stage_us) v = 0;
      const int64_t n0 = c->rep_seq > 24 ? c->rep_seq - 24 : 0;
      const double z = c->trc[n0 % tr_ctx::TRN][0];
      for (int64_t q = n0; q < c->rep_seq; ++q) {
        const double* r = c->trc[q % tr_ctx::TRN];
        fprintf(stderr, "trace %4lld  enq %8.1f exp +%5.1f stage +%5.1f dd +%5.1f | ready %8.1f "
                "replayed %8.1f committed %8.1f\n", (long long)q, r[0] - z, r[1] - r[0], r[2] - r[1],
                r[3] - r[2], r[5] - z, r[6] - z, r[4] - z);
      }
    }
    if (c->timing) {
      memcpy(c->run_us, c->t_us, sizeof(c->t_us));
      memcpy(c->run_nn, c->nn_us, sizeof(c->nn_us));
      harvest_all_side(c);
      harvest_all_main(c);
      if (c->ts_n) {                   // averages over every staged sweep of the run
        c->run_nn[0] = (c->ts_sum[0] + c->ts_sum[1]) / (double)c->ts_n;
        c->run_nn[2] = c->ts_sum[0] / (double)c->ts_n;
      }
    }
    return rc;
  })
}

int tr_last_run_stats(const tr_ctx* c, double* us11, int64_t* commits) {
  if (!c || !us11 || !commits) return fail(TR_E_ARG, "NULL argument");
  memcpy(us11, c->run_us, 5 * sizeof(double));
  memcpy(us11 + 5, c->run_nn, 3 * sizeof(double));
  for (int q = 0; q < 3; ++q) us11[8 + q] = c->run_n ? c->run_host[q] / (double)c->run_n : 0.0;
  *commits = c->run_n;
  return TR_OK;
}

int tr_last_run_kernel_us(const tr_ctx* c, double* us5, int64_t* samples2) {
  if (!c || !us5 || !samples2) return fail(TR_E_ARG, "NULL argument");
  const double ns = c->ts_n ? (double)c->ts_n : 1.0, nm = c->tm_n ? (double)c->tm_n : 1.0;
  us5[0] = c->ts_sum[0] / ns;          // side stream: k_nn_pass1, or the cell lists' build launches
  us5[1] = c->ts_sum[1] / ns;          // k_nn_resolve, or k_nn_grid
  us5[2] = c->tm_sum[0] / nm;          // k_nn_delta (main stream)
  us5[3] = c->tm_sum[1] / nm;          // k_expand_arc
  us5[4] = c->tm_sum[2] / nm;          // dedupe launches
  samples2[0] = c->ts_n;
  samples2[1] = c->tm_n;
  return TR_OK;
}

int tr_rrt_step(tr_ctx* c, const double* gauss, int64_t B, int on_dev, int64_t* n_nodes,
                int64_t* sol) {
  if (!c || !c->session) return fail(TR_E_STATE, "no RRT session: call tr_rrt_begin");
  if (B < 0 || (B && !gauss) || !n_nodes || !sol) return fail(TR_E_ARG, "bad step");
  if (c->r_count) return fail(TR_E_STATE, "tr_rrt_step with pipelined batches in flight");
  if (set_dev(c)) return TR_E_HIP;
  HIPCHK(c->samp.reserve(std::max<int64_t>(B, 1)));
  HIPCHK(c->rec.reserve(std::max<int64_t>(B, 1)));
  const double* dg = gauss;
  if (!on_dev && B) {
    HIPCHK(c->gauss.reserve(3 * B));
    HIPCHK(hipMemcpyAsync(c->gauss.p, gauss, sizeof(double) * 3 * B, hipMemcpyHostToDevice, c->st));
    dg = c->gauss.p;
  }
  if (B) {
    if (int e = tr_rrt_pipe_expand(c, dg, B, c->samp.p, c->rec.p)) return e;
  }
  if (int e = tr_rrt_pipe_dedupe(c, c->samp.p, c->rec.p, B)) return e;
  return tr_rrt_pipe_commit(c, n_nodes, sol);
}

}  // extern "C"

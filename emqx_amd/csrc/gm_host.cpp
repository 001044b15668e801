// gm_host.cpp — emqx_gm_match on HOST buffers: the drop-in path a NIF takes.
//
// The reference matches in the publisher's own process on host data
// (emqx_router:match_routes/1, apps/emqx/src/emqx_router.erl:128-145), so the
// boundary hands over host topics and expects host rows back.  The batch is
// cut into chunks (256K..4M topics, <= 512 MiB of text each) that flow
// through four slots so that PCIe in, the match kernels and PCIe out of
// consecutive chunks overlap:
//
//   worker threads   stage chunk i+2: validate offsets, copy text, each
//                    topic's length as u16 (2 B/topic over PCIe instead of 8:
//                    MQTT topics are at most 65,535 bytes, emqx_topic.erl:45;
//                    a chunk holding a longer one goes as u32 offsets) into
//                    pinned memory
//   h2d stream       pinned -> device                       (chunk i+1)
//   ctx stream       u16 lengths -> u64 offsets (a scan), the device match
//                    (run_match), row offsets back to u32    (chunk i)
//   d2h stream       rows -> pinned                          (chunk i)
//   worker threads   unpack rows into the caller-visible CSR: u64 offsets
//                    rebased by the rows of earlier chunks, ids copied
//                                                            (chunk i-1)
//
// Nothing pageable crosses PCIe and no host thread copies more than its share.
// The result is the same CSR run_match returns (malloc'd, freed by
// emqx_gm_csr_free), so the rows are bit-identical to the device-buffer path.
#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <future>
#include <memory>
#include <queue>
#include <thread>

#include "gm_internal.h"

namespace gm {

namespace {

class Workers {
 public:
  explicit Workers(unsigned n) {
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return unsigned(th_.size()); }
  std::future<void> submit(std::function<void()> f) {
    auto task = std::make_shared<std::packaged_task<void()>>(std::move(f));
    std::future<void> fut = task->get_future();
    {
      std::lock_guard<std::mutex> l(m_);
      q_.push([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop();
      }
      f();
    }
  }
  std::vector<std::thread> th_;
  std::queue<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct Pinned {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t b) {
    if (b <= cap) return true;
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t nb = std::max(b, size_t(1) << 20);
    if (hipHostMalloc(&p, nb, hipHostMallocPortable) != hipSuccess) return false;
    cap = nb;
    return true;
  }
  ~Pinned() {
    if (p) hipHostFree(p);
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

struct Device {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t b) {
    if (b <= cap) return true;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t nb = std::max(b, size_t(1) << 20);
    if (hipMalloc(&p, nb) != hipSuccess) return false;
    cap = nb;
    return true;
  }
  ~Device() {
    if (p) hipFree(p);
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

constexpr int SLOTS = 4;

struct Slot {
  Pinned in_b, in_l, in_o, out_o, out_i;  // text, u16 lengths (u32 offsets: fallback) in; u32 row offsets, ids out
  Device d_b, d_l16, d_o32, d_o64, d_r32;  // text, lengths u16 (offsets u32) -> offsets u64 in; row offsets u32 out
  std::atomic<int> long_topic{0};          // staging met a topic of more than 65,535 bytes
  bool use32 = false;                      // this chunk goes up as u32 offsets
  hipEvent_t h2d = nullptr, comp = nullptr, d2h = nullptr;
  std::vector<std::future<void>> stage_f;  // this slot's staging (run_host_pipe)
  std::vector<std::future<void>> out_f;    // this slot's last unpack
  emqx_gm_csr csr{};                       // device rows of the chunk in flight
  void* call = nullptr;                    // its match call until waited (run_host_pipe)
  bool d2h_pending = false;                // its rows' copy-out is queued (run_host_pipe)
  uint64_t c0 = 0, nc = 0, nbytes = 0, nnz = 0;
};

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* e = knob(name);
  return e ? strtoull(e, nullptr, 10) : dflt;
}

void join(std::vector<std::future<void>>& fs) {
  for (auto& f : fs)
    if (f.valid()) f.get();
  fs.clear();
}

// Worker-side staging of topics [a, e) of the chunk [c0, c0 + nc): offsets
// validated (monotone, inside the chunk's text), each topic's length as u16
// into l -- MQTT caps a topic at 65,535 bytes (apps/emqx/src/emqx_topic.erl:
// 45, MAX_TOPIC_LEN); a longer one (the ABI takes any) sets long_topic and the
// chunk goes up as u32 offsets (stage_off32) -- and the text copied into b
// (nullptr: sent from where it lies), with the chunk's 64 B of padding zeroed.
void stage_part(const uint8_t* tb, const uint64_t* to, uint64_t c0, uint64_t nc, uint64_t a, uint64_t e, uint16_t* l,
                uint8_t* b, std::atomic<int>& bad, std::atomic<int>& long_topic) {
  const uint64_t b0 = to[c0], b1 = to[c0 + nc];
  uint64_t lng = 0;
  for (uint64_t j = a; j < e; ++j) {
    if (to[j + 1] < to[j]) {
      bad.store(1);
      return;
    }
    const uint64_t len = to[j + 1] - to[j];
    lng |= len >> 16;
    l[j - c0] = uint16_t(len);
  }
  if (lng) long_topic.store(1);
  if (to[a] < b0 || to[e] > b1) {  // inside the chunk's text (the chunk plan checked b0 <= b1)
    bad.store(1);
    return;
  }
  if (b && e > a) std::memcpy(b + (to[a] - b0), tb + to[a], to[e] - to[a]);
  if (b && e == c0 + nc) std::memset(b + (to[e] - b0), 0, 64);
}
// the fallback: the chunk's offsets as u32, chunk-relative (validated by stage_part)
void stage_off32(const uint64_t* to, uint64_t c0, uint64_t nc, uint32_t* o) {
  const uint64_t b0 = to[c0];
  for (uint64_t j = 0; j <= nc; ++j) o[j] = uint32_t(to[c0 + j] - b0);
}

}  // namespace

// A staged chunk to its device on stream h: the text (from the pinned staging,
// which holds the 64 B of padding, or -- text != nullptr -- straight from the
// caller's page-locked buffer, the padding zeroed on the device) and its u16
// lengths, or its u32 offsets when a topic was longer than 65,535 bytes.
hipError_t send_in(Slot& s, const uint64_t* to, const uint8_t* text, hipStream_t h) {
  hipError_t e;
  if (!text) {
    e = hipMemcpyAsync(s.d_b.p, s.in_b.p, s.nbytes + 64, hipMemcpyHostToDevice, h);
  } else {
    e = s.nbytes ? hipMemcpyAsync(s.d_b.p, text, s.nbytes, hipMemcpyHostToDevice, h) : hipSuccess;
    if (e == hipSuccess) e = hipMemsetAsync(s.d_b.as<uint8_t>() + s.nbytes, 0, 64, h);
  }
  s.use32 = s.long_topic.load() != 0 || env_u64("GM_HOST_OFF32", 0) != 0;
  if (e == hipSuccess && s.use32) {
    if (!s.in_o.reserve((s.nc + 1) * 4) || !s.d_o32.reserve((s.nc + 1) * 4)) return hipErrorOutOfMemory;
    hipEventSynchronize(s.h2d);  // (the slot's previous send has read in_o)
    stage_off32(to, s.c0, s.nc, s.in_o.as<uint32_t>());
    e = hipMemcpyAsync(s.d_o32.p, s.in_o.p, (s.nc + 1) * 4, hipMemcpyHostToDevice, h);
  } else if (e == hipSuccess) {
    e = hipMemcpyAsync(s.d_l16.p, s.in_l.p, s.nc * 2, hipMemcpyHostToDevice, h);
  }
  if (e == hipSuccess) e = hipEventRecord(s.h2d, h);
  return e;
}
// the chunk's u64 offsets on the device (stream st: the context's), from what send_in sent
int offsets_in(emqx_gm_ctx* c, hipStream_t st, Slot& s) {
  if (s.use32) return launch_off32_to_64(st, s.d_o32.as<uint32_t>(), s.nc + 1, s.d_o64.as<uint64_t>());
  return scan_len16(c, st, s.d_l16.as<uint16_t>(), s.nc, s.d_o64.as<uint64_t>());
}

struct HostPipe {
  int device = 0;
  hipStream_t h2d = nullptr, d2h = nullptr;
  Slot slot[SLOTS];
  std::unique_ptr<Workers> w;
};

void free_host_pipe(emqx_gm_ctx* ctx) {
  HostPipe* hp = ctx->host;
  if (!hp) return;
  hipSetDevice(hp->device);
  for (auto& s : hp->slot) {
    join(s.out_f);
    for (hipEvent_t e : {s.h2d, s.comp, s.d2h})
      if (e) hipEventDestroy(e);
  }
  if (hp->h2d) hipStreamDestroy(hp->h2d);
  if (hp->d2h) hipStreamDestroy(hp->d2h);
  delete hp;
  ctx->host = nullptr;
}

static int host_pipe(emqx_gm_ctx* ctx, HostPipe** out, bool workers = true) {
  if (!ctx->host) {
    auto* hp = new HostPipe;
    hp->device = ctx->device;
    ctx->host = hp;
    hipSetDevice(ctx->device);
    if (hipStreamCreateWithFlags(&hp->h2d, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&hp->d2h, hipStreamNonBlocking) != hipSuccess)
      return set_err(ctx, EMQX_GM_EDEVICE, "match: host pipe streams");
    for (auto& s : hp->slot)
      for (hipEvent_t* e : {&s.h2d, &s.comp, &s.d2h})
        if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess)
          return set_err(ctx, EMQX_GM_EDEVICE, "match: host pipe events");
  }
  if (workers && !ctx->host->w) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    ctx->host->w.reset(new Workers(unsigned(std::max<uint64_t>(1, env_u64("GM_HOST_THREADS", std::min(16u, hw))))));
  }
  *out = ctx->host;
  return 0;
}

// One device, the chunks matched one after another (run_match per chunk, its
// rows unpacked by the workers).  The path of a one-chunk call (the small
// batches a NIF sends): its rows' copy-out rides the call's one host round
// trip (MatchTail); GM_HOST_PIPE=serial forces it for any batch (A/B).
static int run_host_serial(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to,
                           uint64_t n, uint32_t flags, emqx_gm_csr* out) {
  HostPipe* hp = nullptr;
  int rc = host_pipe(ctx, &hp);
  if (rc) return rc;
  Workers& W = *hp->w;
  // chunks: ~6 per call (so PCIe in, the kernels and PCIe out overlap) of
  // 256K..4M topics; GM_HOST_CHUNK pins the size (tests)
  const uint64_t CH = std::max<uint64_t>(
      1024, env_u64("GM_HOST_CHUNK", std::min<uint64_t>(4u << 20, std::max<uint64_t>(256u << 10, n / 6))));
  const uint64_t CB = 512ull << 20;
  const unsigned T = W.size();

  // the caller-visible result (from the context's host pool: emqx_gm_csr_free hands it back)
  uint64_t* r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8));
  uint64_t ids_cap = std::max<uint64_t>(1024, n * 4);
  uint32_t* r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(ids_cap * 4));
  if (!r_off || !r_ids) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return set_err(ctx, EMQX_GM_ENOMEM, "match: host result");
  }
  emqx_gm_match_stats tot{};
  tot.n_topics = n;
  std::vector<std::future<void>> stage_f;
  std::atomic<int> bad{0};
  uint64_t base = 0;  // rows of the chunks before the current one
  int prev = -1;      // slot of the previous chunk (its device rows are released once copied out)

  auto fail = [&](int code, const char* msg) {
    join(stage_f);
    for (auto& s : hp->slot) join(s.out_f);
    hipStreamSynchronize(hp->h2d);
    hipStreamSynchronize(ctx->stream);
    hipStreamSynchronize(hp->d2h);
    for (auto& s : hp->slot)
      if (s.csr.row_off || s.csr.ids) {
        ctx->pool->release(s.csr.row_off);
        ctx->pool->release(s.csr.ids);
        s.csr = emqx_gm_csr{};
      }
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return msg ? set_err(ctx, code, msg) : code;  // nullptr: keep the message of the failing step
  };

  // chunk i = topics [c0, c1): at most CH topics and CB bytes (at least one topic)
  auto plan = [&](uint64_t c0, uint64_t* c1) -> bool {
    uint64_t lo = c0 + 1, hi = std::min(n, c0 + CH);
    if (to[hi] < to[c0] || to[lo] < to[c0]) return false;
    if (to[hi] - to[c0] > CB) {
      while (lo < hi) {  // largest c1 with the chunk's text <= CB
        const uint64_t m = (lo + hi + 1) / 2;
        if (to[m] >= to[c0] && to[m] - to[c0] <= CB) lo = m;
        else hi = m - 1;
      }
      hi = lo;
    }
    *c1 = hi;
    return to[hi] >= to[c0] && to[hi] - to[c0] < (1ull << 32);
  };

  // worker-side staging of chunk [c0, c1) into slot s: offsets checked, u16
  // lengths, text copied, 64 zero bytes of padding (the tokenizer's slack)
  auto stage = [&](Slot& s) {
    const uint64_t c0 = s.c0, nc = s.nc;
    uint16_t* l = s.in_l.as<uint16_t>();
    uint8_t* b = s.in_b.as<uint8_t>();
    s.long_topic.store(0);
    std::atomic<int>* lt = &s.long_topic;
    const uint64_t parts = nc < 65536 ? 1 : T;
    for (uint64_t p = 0; p < parts; ++p) {
      const uint64_t a = c0 + nc * p / parts, e = c0 + nc * (p + 1) / parts;
      auto job = [=, &bad] { stage_part(tb, to, c0, nc, a, e, l, b, bad, *lt); };
      if (parts == 1) job();
      else stage_f.push_back(W.submit(job));
    }
  };

  // chunk boundaries (plan() validates the offsets it relies on)
  std::vector<uint64_t> cb{0};
  while (cb.back() < n) {
    uint64_t c1 = 0;
    if (!plan(cb.back(), &c1)) return fail(EMQX_GM_EINVAL, "match: topic offsets not monotone");
    cb.push_back(c1);
  }
  const int m = int(cb.size()) - 1;
  // input side of a slot: pinned text/offsets -> device text/offsets (busy from
  // staging until its chunk is matched); output side: device row offsets ->
  // pinned rows (busy until its unpack ran).  Chunk i+2 is staged while i+1
  // crosses PCIe and i is matched, so the h2d stream never waits for the CPU.
  auto begin_chunk = [&](int i) -> int {
    Slot& s = hp->slot[i % SLOTS];
    join(s.out_f);               // the slot's last unpack has read its pinned rows
    hipEventSynchronize(s.h2d);  // and its last send has read its pinned input
    s.c0 = cb[i];
    s.nc = cb[i + 1] - cb[i];
    s.nbytes = to[cb[i + 1]] - to[cb[i]];
    if (!s.in_b.reserve(s.nbytes + 64) || !s.in_l.reserve(s.nc * 2 + 2) || !s.d_b.reserve(s.nbytes + 64) ||
        !s.d_l16.reserve(s.nc * 2 + 2) || !s.d_o64.reserve((s.nc + 1) * 8) || !s.d_r32.reserve((s.nc + 1) * 4) ||
        !s.out_o.reserve((s.nc + 1) * 4))
      return EMQX_GM_ENOMEM;
    stage(s);
    return 0;
  };
  auto send_chunk = [&](int i) -> int {
    Slot& s = hp->slot[i % SLOTS];
    join(stage_f);
    if (bad.load()) return EMQX_GM_EINVAL;
    const hipError_t e = send_in(s, to, nullptr, hp->h2d);
    return e == hipSuccess ? 0 : e == hipErrorOutOfMemory ? EMQX_GM_ENOMEM : EMQX_GM_EDEVICE;
  };
  auto pipe_err = [](int code) {
    return code == EMQX_GM_EINVAL ? "match: topic offsets not monotone"
                                  : code == EMQX_GM_ENOMEM ? "match: pinned staging" : "match: host pipe copy";
  };
  if (m > 0 && ((rc = begin_chunk(0)) || (rc = send_chunk(0)))) return fail(rc, pipe_err(rc));
  if (m > 1 && (rc = begin_chunk(1))) return fail(rc, pipe_err(rc));
  for (int i = 0; i < m; ++i) {
    Slot& s = hp->slot[i % SLOTS];
    if (i + 1 < m && (rc = send_chunk(i + 1))) return fail(rc, pipe_err(rc));  // queued behind chunk i's send
    if (i + 2 < m && (rc = begin_chunk(i + 2))) return fail(rc, pipe_err(rc));  // staged on the workers meanwhile
    // match chunk i on the context's stream once its text is on the device
    if (hipStreamWaitEvent(ctx->stream, s.h2d, 0) != hipSuccess || offsets_in(ctx, ctx->stream, s))
      return fail(EMQX_GM_EDEVICE, "match: offsets to device");
    s.csr = emqx_gm_csr{};
    // a one-chunk call queues the rows' copy-out behind the speculative assembly,
    // inside run_match's one host round trip (no second round trip for the rows)
    MatchTail tail;
    const bool one = m == 1 && env_u64("GM_HOST_WIDE_ROWS", 0) == 0;
    if (one)
      tail.enqueue = [&](const uint64_t* d_ro, const uint32_t* d_ids, uint64_t cap) -> int {
        if (!s.out_i.reserve(cap * 4 + 4)) return set_err(ctx, EMQX_GM_ENOMEM, "match: pinned rows");
        if (launch_off64_to_32(ctx->stream, d_ro, s.nc + 1, s.d_r32.as<uint32_t>()) ||
            hipMemcpyAsync(s.out_o.p, s.d_r32.p, (s.nc + 1) * 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            (cap && hipMemcpyAsync(s.out_i.p, d_ids, cap * 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) ||
            hipEventRecord(s.d2h, ctx->stream) != hipSuccess)
          return set_err(ctx, EMQX_GM_EDEVICE, "match: rows to host");
        return 0;
      };
    rc = run_match(ctx, idx, s.d_b.as<uint8_t>(), s.d_o64.as<uint64_t>(), s.nc, flags | EMQX_GM_DEVICE_IO, &s.csr,
                   one ? &tail : nullptr);
    if (rc) return fail(rc, nullptr);
    const emqx_gm_match_stats& cs = ctx->stats;
    tot.nnz += cs.nnz;
    tot.n_overflow += cs.n_overflow;
    tot.n_wildcard_topics += cs.n_wildcard_topics;
    tot.probes += cs.probes;
    tot.match_kernel_ms += cs.match_kernel_ms;
    tot.total_device_ms += cs.total_device_ms;
    s.nnz = s.csr.nnz;
    // row offsets cross PCIe as u32 unless the chunk's rows hold 2^32 ids or more
    // (slow-path rows of thousands of filters): then as they are, u64
    const bool wide = s.nnz > 0xFFFFFFFFull || env_u64("GM_HOST_WIDE_ROWS", 0) != 0;  // (tests force it)
    if (!tail.used) {  // the rows are still on the device
      if ((!wide && launch_off64_to_32(ctx->stream, s.csr.row_off, s.nc + 1, s.d_r32.as<uint32_t>())) ||
          hipEventRecord(s.comp, ctx->stream) != hipSuccess)
        return fail(EMQX_GM_EDEVICE, "match: row offsets");
      // rows back to pinned memory on the d2h stream
      if (!s.out_i.reserve(s.nnz * 4 + 4) || !s.out_o.reserve((s.nc + 1) * (wide ? 8 : 4)))
        return fail(EMQX_GM_ENOMEM, "match: pinned rows");
      if (hipStreamWaitEvent(hp->d2h, s.comp, 0) != hipSuccess ||
          hipMemcpyAsync(s.out_o.p, wide ? static_cast<void*>(s.csr.row_off) : s.d_r32.p, (s.nc + 1) * (wide ? 8 : 4),
                         hipMemcpyDeviceToHost, hp->d2h) != hipSuccess ||
          (s.nnz && hipMemcpyAsync(s.out_i.p, s.csr.ids, s.nnz * 4, hipMemcpyDeviceToHost, hp->d2h) != hipSuccess) ||
          hipEventRecord(s.d2h, hp->d2h) != hipSuccess)
        return fail(EMQX_GM_EDEVICE, "match: rows to host");
    }
    // the previous chunk's device rows are in pinned memory once its d2h event fires
    if (prev >= 0) {
      Slot& p = hp->slot[prev];
      hipEventSynchronize(p.d2h);
      ctx->pool->release(p.csr.row_off);
      ctx->pool->release(p.csr.ids);
      p.csr = emqx_gm_csr{};
    }
    // unpack chunk i into the result on the workers
    if (base + s.nnz > ids_cap) {
      for (auto& q : hp->slot) join(q.out_f);  // nobody writes r_ids while it moves
      while (ids_cap < base + s.nnz) ids_cap *= 2;
      uint32_t* g = static_cast<uint32_t*>(ctx->hpool->alloc(ids_cap * 4));
      if (!g) return fail(EMQX_GM_ENOMEM, "match: host result grow");
      if (base) std::memcpy(g, r_ids, base * 4);
      ctx->hpool->release(r_ids);
      r_ids = g;
    }
    {
      const uint64_t parts = s.nc < 65536 ? 1 : T;
      const uint32_t* ro = s.out_o.as<uint32_t>();
      const uint64_t* ro64 = s.out_o.as<uint64_t>();
      const uint32_t* ri = s.out_i.as<uint32_t>();
      const hipEvent_t ev = s.d2h;
      const uint64_t sc0 = s.c0, snc = s.nc, sbase = base;
      uint32_t* dst_ids = r_ids;
      for (uint64_t p = 0; p < parts; ++p) {
        const uint64_t a = snc * p / parts, e = snc * (p + 1) / parts;
        auto unpack = [=] {
          hipEventSynchronize(ev);
          auto row = [&](uint64_t j) -> uint64_t { return wide ? ro64[j] : uint64_t(ro[j]); };
          for (uint64_t j = a; j < e; ++j) r_off[sc0 + j] = sbase + row(j);
          if (e > a) std::memcpy(dst_ids + sbase + row(a), ri + row(a), (row(e) - row(a)) * 4);
        };
        // a call of one small chunk unpacks on the calling thread (no hand-off to a
        // worker: nothing else is in flight to overlap with)
        if (m == 1 && parts == 1) unpack();
        else s.out_f.push_back(W.submit(unpack));
      }
    }
    base += s.nnz;
    prev = i % SLOTS;
  }
  for (auto& q : hp->slot) join(q.out_f);
  if (prev >= 0) {
    Slot& p = hp->slot[prev];
    hipEventSynchronize(p.d2h);
    ctx->pool->release(p.csr.row_off);
    ctx->pool->release(p.csr.ids);
    p.csr = emqx_gm_csr{};
  }
  r_off[n] = base;
  if (n == 0) r_off[0] = 0;
  tot.nnz = base;
  ctx->stats = tot;
  out->n_rows = n;
  out->nnz = base;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;  // the owning context (emqx_gm_csr_free checks it)
  return 0;
}

// The pipelined path: the chunks of one call spread over the context's
// devices (chunk i on device i mod K, K = 1 + the members the index has
// replicas on), each device with its own streams and slots, up to
// PIPE_DEPTH chunks in flight per device.  Per chunk:
//   workers      offsets validated and rebased to u32 (and the text copied
//                into pinned staging, unless it already lies in an
//                emqx_gm_host_alloc buffer: then it is sent from there)
//   h2d stream   text + offsets to the device
//   ctx stream   u32 -> u64 offsets, the match call queued (match_submit)
//   host         the call waited for IN BATCH ORDER (match_wait), so the
//                rows before it are known: its base
//   d2h stream   row offsets + base (on the device), then rows and ids by
//                DMA straight into the caller's result at their final place
//                -- the result is page-locked (the context's host pool), so
//                no host thread copies a row
// A result that cannot be page-locked falls back to pinned bounce buffers
// unpacked by the workers (the serial path's way).
constexpr int PIPE_DEPTH = 2;

static int run_host_pipe(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to,
                         uint64_t n, uint32_t flags, const std::vector<emqx_gm_ctx*>& mem,
                         const std::vector<const emqx_gm_index*>& rix, const std::vector<uint64_t>& cb,
                         emqx_gm_csr* out) {
  const int K = int(mem.size());
  const int m = int(cb.size()) - 1;
  // every member device for the whole call: its host pipeline, pools and
  // stream are also what a small call on that device alone uses (gm_api.cpp
  // match_small holds only the member's lock).  Order: the first device's lock
  // (the caller's), then the members' in order; a small call takes one member's.
  std::vector<std::unique_lock<std::recursive_mutex>> held;
  for (int k = 1; k < K; ++k) held.emplace_back(mem[k]->mu);
  std::vector<HostPipe*> hps(K);
  for (int k = 0; k < K; ++k)
    if (int rc = host_pipe(mem[k], &hps[k], k == 0)) return rc;
  hipSetDevice(ctx->device);
  Workers& W = *hps[0]->w;
  const unsigned T = W.size();
  const bool direct_in = host_pinned_range(tb + to[0], to[n] - to[0]);
  // the caller-visible result, page-locked when the host allows it
  uint64_t ids_cap = std::max<uint64_t>(1024, uint64_t(double(n) * std::max(4.0, 1.25 * ctx->ids_per_topic)));
  // (GM_HOST_BOUNCE / GM_HOST_WIDE_ROWS: the bounce-buffer output, the latter
  // with u64 row offsets over PCIe -- tests and A/Bs)
  const bool wide_rows = env_u64("GM_HOST_WIDE_ROWS", 0) != 0;
  bool direct_out = !env_u64("GM_HOST_BOUNCE", 0) && !wide_rows;
  uint64_t* r_off = nullptr;
  uint32_t* r_ids = nullptr;
  if (direct_out) {
    r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8, true));
    r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(ids_cap * 4, true));
    if (!r_off || !r_ids) {
      ctx->hpool->release(r_off);
      ctx->hpool->release(r_ids);
      r_off = nullptr;
      r_ids = nullptr;
      direct_out = false;
    }
  }
  if (!direct_out) {
    r_off = static_cast<uint64_t*>(ctx->hpool->alloc((n + 1) * 8));
    r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(ids_cap * 4));
  }
  if (!r_off || !r_ids) {
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return set_err(ctx, EMQX_GM_ENOMEM, "match: host result");
  }
  auto dev_of = [&](int i) { return i % K; };
  auto slot_of = [&](int i) -> Slot& { return hps[i % K]->slot[(i / K) % SLOTS]; };
  std::atomic<int> bad{0};
  emqx_gm_match_stats tot{};
  tot.n_topics = n;
  uint64_t base = 0;

  // a slot's previous chunk done: its copy-out landed, its unpack ran, its device rows back to the pool
  auto retire = [&](int k, Slot& s) {
    join(s.stage_f);
    if (s.call) {  // (an abandoned call: only on the failure path)
      emqx_gm_csr c{};
      hipSetDevice(mem[k]->device);
      (void)match_wait(mem[k], s.call, &c);
      s.call = nullptr;
      if (c.row_off || c.ids) s.csr = c;
    }
    if (s.d2h_pending) {
      hipEventSynchronize(s.d2h);
      s.d2h_pending = false;
    }
    join(s.out_f);
    if (s.csr.row_off || s.csr.ids) {
      mem[k]->pool->release(s.csr.row_off);
      mem[k]->pool->release(s.csr.ids);
      s.csr = emqx_gm_csr{};
    }
  };
  auto fail = [&](int code, const char* msg) {
    for (int k = 0; k < K; ++k) {
      for (auto& s : hps[k]->slot) retire(k, s);
      hipSetDevice(mem[k]->device);
      hipStreamSynchronize(hps[k]->h2d);
      hipStreamSynchronize(mem[k]->stream);
      hipStreamSynchronize(hps[k]->d2h);
    }
    hipSetDevice(ctx->device);
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return msg ? set_err(ctx, code, msg) : code;  // nullptr: keep the message of the failing step
  };

  // chunk i's staging: the slot retired, buffers sized, the worker jobs queued
  auto stage = [&](int i) -> int {
    const int k = dev_of(i);
    Slot& s = slot_of(i);
    retire(k, s);
    hipSetDevice(mem[k]->device);
    hipEventSynchronize(s.h2d);  // (its last send has read the pinned input)
    s.c0 = cb[i];
    s.nc = cb[i + 1] - cb[i];
    s.nbytes = to[cb[i + 1]] - to[cb[i]];
    if ((!direct_in && !s.in_b.reserve(s.nbytes + 64)) || !s.in_l.reserve(s.nc * 2 + 2) ||
        !s.d_b.reserve(s.nbytes + 64) || !s.d_l16.reserve(s.nc * 2 + 2) || !s.d_o64.reserve((s.nc + 1) * 8) ||
        (!direct_out && (!s.d_r32.reserve((s.nc + 1) * 4) || !s.out_o.reserve((s.nc + 1) * 4)))) {
      hipSetDevice(ctx->device);
      return EMQX_GM_ENOMEM;
    }
    hipSetDevice(ctx->device);
    const uint64_t c0 = s.c0, nc = s.nc;
    uint16_t* l = s.in_l.as<uint16_t>();
    uint8_t* b = direct_in ? nullptr : s.in_b.as<uint8_t>();
    s.long_topic.store(0);
    std::atomic<int>* lt = &s.long_topic;
    const uint64_t parts = nc < 65536 ? 1 : T;
    for (uint64_t p = 0; p < parts; ++p) {
      const uint64_t a = c0 + nc * p / parts, e = c0 + nc * (p + 1) / parts;
      s.stage_f.push_back(W.submit([=, &bad] { stage_part(tb, to, c0, nc, a, e, l, b, bad, *lt); }));
    }
    return 0;
  };
  // chunk i to its device (h2d stream)
  auto send = [&](int i) -> int {
    const int k = dev_of(i);
    Slot& s = slot_of(i);
    join(s.stage_f);
    if (bad.load()) return EMQX_GM_EINVAL;
    hipSetDevice(mem[k]->device);
    const hipError_t e = send_in(s, to, direct_in ? tb + to[s.c0] : nullptr, hps[k]->h2d);
    hipSetDevice(ctx->device);
    return e == hipSuccess ? 0 : e == hipErrorOutOfMemory ? EMQX_GM_ENOMEM : EMQX_GM_EDEVICE;
  };
  // chunk i's match queued on its device
  auto submit = [&](int i) -> int {
    const int k = dev_of(i);
    Slot& s = slot_of(i);
    emqx_gm_ctx* mc = mem[k];
    hipSetDevice(mc->device);
    int rc = 0;
    {
      std::lock_guard<std::recursive_mutex> lk(mc->mu);
      if (hipStreamWaitEvent(mc->stream, s.h2d, 0) != hipSuccess || offsets_in(mc, mc->stream, s))
        rc = set_err(ctx, EMQX_GM_EDEVICE, "match: offsets to device");
      else
        rc = match_submit(mc, rix[k], s.d_b.as<uint8_t>(), s.d_o64.as<uint64_t>(), s.nc, flags | EMQX_GM_DEVICE_IO,
                          &s.call);
    }
    hipSetDevice(ctx->device);
    return rc;
  };
  // chunk i waited for (batch order), its rows sent to their place in the result
  auto finish = [&](int i) -> int {
    const int k = dev_of(i);
    Slot& s = slot_of(i);
    emqx_gm_ctx* mc = mem[k];
    hipSetDevice(mc->device);
    void* call = s.call;
    s.call = nullptr;
    int rc = match_wait(mc, call, &s.csr);
    if (rc) {
      hipSetDevice(ctx->device);
      return rc;
    }
    const emqx_gm_match_stats& cs = mc->stats;
    tot.nnz += cs.nnz;
    tot.n_overflow += cs.n_overflow;
    tot.n_wildcard_topics += cs.n_wildcard_topics;
    tot.probes += cs.probes;
    tot.match_kernel_ms += cs.match_kernel_ms;
    tot.total_device_ms += cs.total_device_ms;
    s.nnz = s.csr.nnz;
    if (base + s.nnz > ids_cap) {  // grow the result: nothing may be writing it meanwhile
      for (int q = 0; q < K; ++q)
        for (auto& z : hps[q]->slot) {
          if (z.d2h_pending) {
            hipEventSynchronize(z.d2h);
            z.d2h_pending = false;
          }
          join(z.out_f);
        }
      uint64_t ncap = ids_cap;
      while (ncap < base + s.nnz) ncap *= 2;
      uint32_t* g = static_cast<uint32_t*>(ctx->hpool->alloc(ncap * 4, direct_out));
      if (!g) {
        hipSetDevice(ctx->device);
        return set_err(ctx, EMQX_GM_ENOMEM, "match: host result grow");
      }
      if (base) std::memcpy(g, r_ids, base * 4);
      ctx->hpool->release(r_ids);
      r_ids = g;
      ids_cap = ncap;
    }
    hipStream_t d = hps[k]->d2h;  // (the call is complete: no event to wait for)
    hipError_t e = hipSuccess;
    if (direct_out) {
      if (launch_add_u64(d, s.csr.row_off, s.nc, base)) e = hipErrorLaunchFailure;
      if (e == hipSuccess)
        e = hipMemcpyAsync(r_off + s.c0, s.csr.row_off, s.nc * 8, hipMemcpyDeviceToHost, d);
      if (e == hipSuccess && s.nnz) e = hipMemcpyAsync(r_ids + base, s.csr.ids, s.nnz * 4, hipMemcpyDeviceToHost, d);
      if (e == hipSuccess) e = hipEventRecord(s.d2h, d);
    } else {
      const bool wide = s.nnz > 0xFFFFFFFFull || wide_rows;
      if (!s.out_i.reserve(s.nnz * 4 + 4) || !s.out_o.reserve((s.nc + 1) * (wide ? 8 : 4))) {
        hipSetDevice(ctx->device);
        return set_err(ctx, EMQX_GM_ENOMEM, "match: pinned rows");
      }
      if (!wide && launch_off64_to_32(d, s.csr.row_off, s.nc + 1, s.d_r32.as<uint32_t>())) e = hipErrorLaunchFailure;
      if (e == hipSuccess)
        e = hipMemcpyAsync(s.out_o.p, wide ? static_cast<void*>(s.csr.row_off) : s.d_r32.p,
                           (s.nc + 1) * (wide ? 8 : 4), hipMemcpyDeviceToHost, d);
      if (e == hipSuccess && s.nnz) e = hipMemcpyAsync(s.out_i.p, s.csr.ids, s.nnz * 4, hipMemcpyDeviceToHost, d);
      if (e == hipSuccess) e = hipEventRecord(s.d2h, d);
      if (e == hipSuccess) {
        const uint64_t parts = s.nc < 65536 ? 1 : T;
        const uint32_t* ro = s.out_o.as<uint32_t>();
        const uint64_t* ro64 = s.out_o.as<uint64_t>();
        const uint32_t* ri = s.out_i.as<uint32_t>();
        const hipEvent_t ev = s.d2h;
        const uint64_t sc0 = s.c0, snc = s.nc, sbase = base;
        uint32_t* dst_ids = r_ids;
        for (uint64_t p = 0; p < parts; ++p) {
          const uint64_t a = snc * p / parts, z = snc * (p + 1) / parts;
          s.out_f.push_back(W.submit([=] {
            hipEventSynchronize(ev);
            auto row = [&](uint64_t j) -> uint64_t { return wide ? ro64[j] : uint64_t(ro[j]); };
            for (uint64_t j = a; j < z; ++j) r_off[sc0 + j] = sbase + row(j);
            if (z > a) std::memcpy(dst_ids + sbase + row(a), ri + row(a), (row(z) - row(a)) * 4);
          }));
        }
      }
    }
    hipSetDevice(ctx->device);
    if (e != hipSuccess) return set_err(ctx, EMQX_GM_EDEVICE, "match: rows to host");
    s.d2h_pending = true;
    base += s.nnz;
    return 0;
  };

  auto pipe_err = [](int code) {
    return code == EMQX_GM_EINVAL ? "match: topic offsets not monotone"
                                  : code == EMQX_GM_ENOMEM ? "match: pinned staging" : "match: host pipe copy";
  };
  int ns = 0, nh = 0, nu = 0;  // next chunk to stage, to send, to submit
  for (int i = 0; i < m; ++i) {
    const int lim = std::min(m, i + K * PIPE_DEPTH);
    while (nu < lim) {
      while (nh <= nu) {
        while (ns < std::min(m, nh + K + 1))
          if (int rc = stage(ns++)) return fail(rc, pipe_err(rc));
        if (int rc = send(nh++)) return fail(rc, pipe_err(rc));
      }
      if (int rc = submit(nu++)) return fail(rc, nullptr);
    }
    if (int rc = finish(i)) return fail(rc, nullptr);
  }
  for (int k = 0; k < K; ++k)
    for (auto& s : hps[k]->slot) retire(k, s);
  hipSetDevice(ctx->device);
  r_off[n] = base;
  tot.nnz = base;
  ctx->stats = tot;
  out->n_rows = n;
  out->nnz = base;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;  // the owning context (emqx_gm_csr_free checks it)
  return 0;
}

// Small host-buffer calls: copies up to this many bytes run as kernels over
// mapped page-locked memory; larger ones on the copy engine (gm_host.cpp A/B,
// profiles/r06_p: at 262,144 C2 topics the mapped copies ran at 0.56x)
constexpr size_t kMappedMax = size_t(1) << 20;
// a page-locked buffer as the device addresses it, for a copy of `bytes` as a kernel (nullptr: the copy engine)
static uint32_t* mapped(void* h, size_t bytes) {
  void* d = nullptr;
  return bytes <= kMappedMax && hipHostGetDevicePointer(&d, h, 0) == hipSuccess ? static_cast<uint32_t*>(d) : nullptr;
}
// one host <-> device copy of a small call: a kernel over mapped memory up to kMappedMax, else the copy engine
static hipError_t small_copy(hipStream_t st, void* dst, const void* src, size_t bytes, bool to_dev) {
  if (!bytes) return hipSuccess;
  uint32_t* hm = mapped(const_cast<void*>(to_dev ? src : dst), bytes);
  if (hm && !(bytes & 3))
    return launch_copy_u32x2(st, to_dev ? hm : static_cast<const uint32_t*>(src),
                             to_dev ? static_cast<uint32_t*>(dst) : hm, bytes / 4, nullptr, nullptr, 0)
               ? hipErrorLaunchFailure
               : hipSuccess;
  return hipMemcpyAsync(dst, src, bytes, to_dev ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, st);
}

// a small host fan-out: at most this many deliveries (its speculative page-locked result)
constexpr uint64_t kFanSmallDeliveries = uint64_t(16) << 20;

uint64_t host_chunk_topics() { return std::max<uint64_t>(1024, env_u64("GM_HOST_CHUNK", 256u << 10)); }

int run_host_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                   uint32_t flags, emqx_gm_csr* out, emqx_gm_match_stats* st_out, SmallFan* fan) {
  // ---- outside the lock: the offsets checked, the call's inputs staged in a
  // page-locked buffer of its own: [text | 64 B of padding | u16 lengths (u32
  // offsets past 65,535 B)] -- past kMappedMax of text already page-locked, the
  // lengths alone (the text goes up from the caller's buffer on the copy engine)
  uint64_t lng = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (to[i + 1] < to[i]) return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
    lng |= (to[i + 1] - to[i]) >> 16;
  }
  const bool use32 = lng != 0 || env_u64("GM_HOST_OFF32", 0) != 0;
  const uint64_t b0 = n ? to[0] : 0, nbytes = n ? to[n] - b0 : 0;
  const bool direct = nbytes > kMappedMax && host_pinned_range(tb + b0, nbytes);
  struct Pin {
    PinPool* pool;
    void* p = nullptr;
    ~Pin() {
      if (p) pool->put(p);
    }
  } pin{ctx->pins};
  const size_t lbytes = use32 ? (n + 1) * 4 : n * 2 + 2;
  const size_t o_len = direct ? 0 : (nbytes + 64 + 255) & ~size_t(255);  // the lengths' offset in the input
  const size_t in_bytes = (o_len + lbytes + 15) & ~size_t(15), obytes = (n + 1) * 8;
  if (!(pin.p = ctx->pins->get(in_bytes))) return set_err(ctx, EMQX_GM_ENOMEM, "match: pinned staging");
  uint8_t* in = static_cast<uint8_t*>(pin.p);
  if (!direct) {
    if (nbytes) std::memcpy(in, tb + b0, nbytes);
    std::memset(in + nbytes, 0, 64);
  }
  if (use32) {
    stage_off32(to, 0, n, reinterpret_cast<uint32_t*>(in + o_len));
  } else {
    uint16_t* l = reinterpret_cast<uint16_t*>(in + o_len);
    for (uint64_t i = 0; i < n; ++i) l[i] = uint16_t(to[i + 1] - to[i]);
  }
  // the page-locked buffers as the device addresses them: up to kMappedMax a copy
  // runs as a kernel on the call's own queue (k_copy_u32x2: no hand-over between
  // the copy engine and the call's kernels, ~10 us each) -- past it, or if a
  // buffer is not mapped, on the copy engine
  const uint32_t* in_dev = mapped(pin.p, in_bytes);
  // ---- under the lock: the inputs up, the call queued (untimed: no timestamps
  // on the stream), its rows' copy-out behind its speculative assembly -- one
  // device round trip for the call
  std::unique_lock<std::recursive_mutex> lk(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  void* dv[3] = {ctx->pool->alloc(in_bytes), ctx->pool->alloc((n + 1) * 8),
                 direct ? ctx->pool->alloc(nbytes + 64) : nullptr};
  auto drop_dev = [&]() {  // (under the lock; the call's work is done or was never queued)
    for (void*& q : dv)
      if (q) ctx->pool->release(q);
  };
  if (!dv[0] || !dv[1] || (direct && !dv[2])) {
    drop_dev();
    return set_err(ctx, EMQX_GM_ENOMEM, "match: input workspace");
  }
  uint8_t* d_b = static_cast<uint8_t*>(direct ? dv[2] : dv[0]);
  const void* d_l = static_cast<uint8_t*>(dv[0]) + o_len;
  uint64_t* d_o = static_cast<uint64_t*>(dv[1]);
  hipError_t e = in_dev ? (launch_copy_u32x2(st, in_dev, static_cast<uint32_t*>(dv[0]), in_bytes / 4, nullptr,
                                             nullptr, 0) ? hipErrorLaunchFailure : hipSuccess)
                        : hipMemcpyAsync(dv[0], in, in_bytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && direct) e = hipMemcpyAsync(d_b, tb + b0, nbytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && direct) e = hipMemsetAsync(d_b + nbytes, 0, 64, st);
  if (e != hipSuccess || (use32 ? launch_off32_to_64(st, static_cast<const uint32_t*>(d_l), n + 1, d_o)
                                : scan_len16(ctx, st, static_cast<const uint16_t*>(d_l), n, d_o))) {
    hipStreamSynchronize(st);
    drop_dev();
    return set_err(ctx, EMQX_GM_EDEVICE, "match: inputs to device");
  }
  // the caller-visible result, page-locked from the context's host pool
  // (emqx_gm_csr_free hands it back): the rows land there straight from the
  // device, behind the call's speculative assembly (the row offsets as they
  // are, u64: one launch fewer)
  uint64_t* r_off = nullptr;
  uint32_t* r_ids = nullptr;
  // fan: the deliveries of the speculative rows, queued behind them into a
  // capacity of their own (this context's recent deliveries per match), their
  // page-locked result filled the same way
  uint64_t* f_off = nullptr;
  uint32_t* f_ids = nullptr;
  uint64_t cap_f = 0;
  auto drop_fan = [&]() {  // (under the lock)
    ctx->hpool->release(f_off);
    ctx->hpool->release(f_ids);
    f_off = nullptr;
    f_ids = nullptr;
  };
  auto drop_res = [&]() {  // (under the lock)
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    r_off = nullptr;
    r_ids = nullptr;
    drop_fan();
  };
  MatchTail tail;
  tail.enqueue = [&](const uint64_t* d_ro, const uint32_t* d_ids, uint64_t cap) -> int {
    r_off = static_cast<uint64_t*>(ctx->hpool->alloc(obytes, true));
    size_t ib = 4096;  // (a power of two: the result buffers come back from the host pool's cache)
    while (ib < cap * 4 + 16) ib <<= 1;
    r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(ib, true));
    if (!r_off || !r_ids) return set_err(ctx, EMQX_GM_ENOMEM, "match: host result");
    uint32_t* off_dev = mapped(r_off, obytes + cap * 4);
    uint32_t* ids_dev = mapped(r_ids, obytes + cap * 4);
    hipError_t x = hipSuccess;
    if (off_dev && ids_dev) {
      if (launch_copy_u32x2(st, reinterpret_cast<const uint32_t*>(d_ro), off_dev, obytes / 4, d_ids, ids_dev, cap,
                            d_ro + n))
        x = hipErrorLaunchFailure;
    } else {
      x = hipMemcpyAsync(r_off, d_ro, obytes, hipMemcpyDeviceToHost, st);
      if (x == hipSuccess && cap) x = hipMemcpyAsync(r_ids, d_ids, cap * 4, hipMemcpyDeviceToHost, st);
    }
    if (x != hipSuccess) return set_err(ctx, EMQX_GM_EDEVICE, "match: rows to host");
    // (cap = 1024 + the topics x recent ids per topic x1.25: the expected rows past the slack)
    const double want = 1024.0 + double(cap > 1024 ? cap - 1024 : 1) * ctx->subs_per_match;
    if (fan) fan->cap = uint64_t(want);
    if (!fan || want > double(kFanSmallDeliveries)) return 0;  // (no fan-out here: the caller runs its own)
    for (cap_f = 1024; double(cap_f) < want;) cap_f <<= 1;
    void* fd[3] = {ctx->pool->alloc((cap + 1) * 8), ctx->pool->alloc(obytes), ctx->pool->alloc(cap_f * 4 + 16)};
    f_off = static_cast<uint64_t*>(ctx->hpool->alloc(obytes, true));
    f_ids = static_cast<uint32_t*>(ctx->hpool->alloc(cap_f * 4 + 16, true));
    if (!fd[0] || !fd[1] || !fd[2] || !f_off || !f_ids) {  // (no room: the caller runs its own fan-out)
      for (void* q : fd)
        if (q) ctx->pool->release(q);
      drop_fan();
      return 0;
    }
    int frc = queue_fanout_spec(ctx, idx, d_ro, d_ids, n, cap, cap_f, static_cast<uint64_t*>(fd[0]),
                                static_cast<uint64_t*>(fd[1]), static_cast<uint32_t*>(fd[2]));
    uint32_t* fo_dev = mapped(f_off, obytes + cap_f * 4);
    uint32_t* fi_dev = mapped(f_ids, obytes + cap_f * 4);
    if (!frc && fo_dev && fi_dev) {
      if (launch_copy_u32x2(st, static_cast<const uint32_t*>(fd[1]), fo_dev, obytes / 4,
                            static_cast<const uint32_t*>(fd[2]), fi_dev, cap_f, static_cast<const uint64_t*>(fd[1]) + n))
        frc = set_err(ctx, EMQX_GM_EDEVICE, "match_fanout: deliveries to host");
    } else if (!frc) {
      if (hipMemcpyAsync(f_off, fd[1], obytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipMemcpyAsync(f_ids, fd[2], cap_f * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        frc = set_err(ctx, EMQX_GM_EDEVICE, "match_fanout: deliveries to host");
    }
    if (frc) {
      hipStreamSynchronize(st);
      for (void* q : fd) ctx->pool->release(q);
      return frc;
    }
    ctx->pool->release_after(fd, 3, st);
    return 0;
  };
  void* ticket = nullptr;
  int rc = match_submit(ctx, idx, d_b, d_o, n, flags | EMQX_GM_DEVICE_IO | EMQX_GM_NO_TIMING, &ticket, &tail);
  if (rc) {
    hipStreamSynchronize(st);
    drop_dev();
    drop_res();
    return rc;
  }
  lk.unlock();
  // ---- outside the lock: the device round trip (other callers queue theirs meanwhile)
  emqx_gm_csr dc{};
  rc = match_wait(ctx, ticket, &dc, &tail, st_out);
  lk.lock();
  drop_dev();  // (match_wait returned: this call's work on them is done)
  if (rc) {
    drop_res();
    return rc;
  }
  const uint64_t nnz = dc.nnz;
  if (!tail.used) {  // past the speculative capacity: the rows copied out now, into a result of their size
    ctx->hpool->release(r_ids);
    if (!r_off) r_off = static_cast<uint64_t*>(ctx->hpool->alloc(obytes));
    r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(nnz * 4 + 4));
    hipError_t x = r_off && r_ids ? hipMemcpyAsync(r_off, dc.row_off, obytes, hipMemcpyDeviceToHost, st)
                                  : hipErrorOutOfMemory;
    if (x == hipSuccess && nnz) x = hipMemcpyAsync(r_ids, dc.ids, nnz * 4, hipMemcpyDeviceToHost, st);
    if (x == hipSuccess) x = hipStreamSynchronize(st);
    if (x != hipSuccess) {
      drop_res();
      ctx->pool->release(dc.row_off);
      ctx->pool->release(dc.ids);
      return set_err(ctx, x == hipErrorOutOfMemory ? EMQX_GM_ENOMEM : EMQX_GM_EDEVICE, "match: host result");
    }
  }
  if (fan) fan->rows_spec = tail.used;
  if (f_off) {  // the fused fan-out holds if the rows were the speculative ones and its deliveries fit
    const uint64_t tot = f_off[n];
    fan->queued = true;
    fan->total = tot;
    fan->cap = cap_f;
    if (tail.used && nnz) ctx->subs_per_match = std::max(1.0, double(tot) / double(nnz));
    if (tail.used && tot <= cap_f) {
      fan->ok = true;
      fan->out = emqx_gm_csr{};
      fan->out.n_rows = n;
      fan->out.nnz = tot;
      fan->out.row_off = f_off;
      fan->out.ids = f_ids;
      fan->out.on_device = 0;
      fan->out.priv = ctx;
    } else {
      drop_fan();
    }
  }
  ctx->pool->release(dc.row_off);
  ctx->pool->release(dc.ids);
  lk.unlock();
  out->n_rows = n;
  out->nnz = nnz;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;  // the owning context (emqx_gm_csr_free checks it)
  return 0;
}


int run_fanout_small(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const emqx_gm_index* host, const emqx_gm_csr* m,
                     emqx_gm_csr* out, emqx_gm_match_stats* st_out) {
  // ---- outside the lock: the rows checked and staged in a page-locked buffer
  // of the call's own: [row offsets | ids]
  // (rows that are not a plain CSR over [0, nnz) take the ordinary path, as they always have)
  const uint64_t n = m->n_rows, nnz = m->nnz, nf = host->view.n_filters;
  if (m->row_off[0] != 0 || m->row_off[n] != nnz) return 1;
  for (uint64_t i = 0; i < n; ++i)
    if (m->row_off[i + 1] < m->row_off[i]) return 1;
  for (uint64_t i = 0; i < nnz; ++i)
    if (m->ids[i] >= nf) return set_err(ctx, EMQX_GM_EINVAL, "fanout: filter id out of range");
  const size_t obytes = (n + 1) * 8, o_ids = (obytes + 15) & ~size_t(15);
  const size_t in_bytes = (o_ids + nnz * 4 + 15) & ~size_t(15);
  struct Pin {
    PinPool* pool;
    void* p = nullptr;
    ~Pin() {
      if (p) pool->put(p);
    }
  } pin{ctx->pins};
  // ---- under the lock: rows up, the deliveries into a speculative capacity
  // (this context's recent deliveries per match x1.25, a power of two: the
  // result buffers come back from the host pool's cache), the result's
  // copy-out straight into the page-locked result (as long as the device's
  // total), the call's end event; the device workspace handed back behind it
  std::unique_lock<std::recursive_mutex> lk(ctx->mu);
  const double want = 1024.0 + double(nnz) * ctx->subs_per_match * 1.25;
  if (want > double(kFanSmallDeliveries)) return 1;  // (a wide fan-out: the ordinary path counts first)
  uint64_t cap = 1024;
  while (double(cap) < want) cap <<= 1;
  lk.unlock();
  if (!(pin.p = ctx->pins->get(in_bytes))) return set_err(ctx, EMQX_GM_ENOMEM, "fanout: pinned staging");
  uint8_t* in = static_cast<uint8_t*>(pin.p);
  std::memcpy(in, m->row_off, obytes);
  if (nnz) std::memcpy(in + o_ids, m->ids, nnz * 4);
  lk.lock();
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  void* dv[4] = {ctx->pool->alloc(in_bytes), ctx->pool->alloc((nnz + 1) * 8), ctx->pool->alloc(obytes),
                 ctx->pool->alloc(cap * 4 + 16)};
  uint64_t* r_off = static_cast<uint64_t*>(ctx->hpool->alloc(obytes, true));
  uint32_t* r_ids = static_cast<uint32_t*>(ctx->hpool->alloc(cap * 4 + 16, true));
  hipEvent_t done = nullptr;
  if (!ctx->ev_free.empty()) {
    done = ctx->ev_free.back();
    ctx->ev_free.pop_back();
  } else if (hipEventCreate(&done) != hipSuccess) {  // (a timing event: the list serves timed match calls too)
    done = nullptr;
  }
  auto fail = [&](int code, const char* msg) {  // (under the lock)
    hipStreamSynchronize(st);
    for (void* q : dv)
      if (q) ctx->pool->release(q);
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    if (done) ctx->ev_free.push_back(done);
    return set_err(ctx, code, msg);
  };
  if (!dv[0] || !dv[1] || !dv[2] || !dv[3] || !r_off || !r_ids) return fail(EMQX_GM_ENOMEM, "fanout: workspace");
  if (!done) return fail(EMQX_GM_EDEVICE, "fanout: event");
  uint8_t* d_in = static_cast<uint8_t*>(dv[0]);
  hipError_t e = small_copy(st, d_in, in, in_bytes, true);
  if (e != hipSuccess) return fail(EMQX_GM_EDEVICE, "fanout: rows to device");
  if (int rc = queue_fanout_small(ctx, idx, reinterpret_cast<const uint64_t*>(d_in),
                                  reinterpret_cast<const uint32_t*>(d_in + o_ids), n, nnz, cap,
                                  static_cast<uint64_t*>(dv[1]), static_cast<uint64_t*>(dv[2]),
                                  static_cast<uint32_t*>(dv[3]))) {
    hipStreamSynchronize(st);
    for (void* q : dv) ctx->pool->release(q);
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    ctx->ev_free.push_back(done);
    return rc;
  }
  const uint64_t* d_total = static_cast<const uint64_t*>(dv[2]) + n;  // the rows' row_off[n]
  uint32_t* off_dev = mapped(r_off, obytes + cap * 4);
  uint32_t* ids_dev = mapped(r_ids, obytes + cap * 4);
  if (off_dev && ids_dev) {
    e = launch_copy_u32x2(st, static_cast<const uint32_t*>(dv[2]), off_dev, obytes / 4,
                          static_cast<const uint32_t*>(dv[3]), ids_dev, cap, d_total)
            ? hipErrorLaunchFailure
            : hipSuccess;
  } else {
    e = hipMemcpyAsync(r_off, dv[2], obytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(r_ids, dv[3], cap * 4, hipMemcpyDeviceToHost, st);
  }
  if (e == hipSuccess) e = hipEventRecord(done, st);
  if (e != hipSuccess) return fail(EMQX_GM_EDEVICE, "fanout: rows to host");
  ctx->pool->release_after(dv, 4, st);
  lk.unlock();
  // ---- outside the lock: the device round trip
  e = hipEventSynchronize(done);
  lk.lock();
  ctx->ev_free.push_back(done);
  const uint64_t total = e == hipSuccess ? r_off[n] : 0;
  if (e == hipSuccess && nnz) ctx->subs_per_match = std::max(1.0, double(total) / double(nnz));
  if (e != hipSuccess || total > cap) {  // (a device fault; or past the capacity: the ordinary path, which counts first)
    ctx->hpool->release(r_off);
    ctx->hpool->release(r_ids);
    return e != hipSuccess ? set_err(ctx, EMQX_GM_EDEVICE, "fanout: device") : 1;
  }
  lk.unlock();
  if (st_out) {
    *st_out = emqx_gm_match_stats{};
    st_out->n_topics = n;
    st_out->nnz = total;
  }
  out->n_rows = n;
  out->nnz = total;
  out->row_off = r_off;
  out->ids = r_ids;
  out->on_device = 0;
  out->priv = ctx;  // the owning context (emqx_gm_csr_free checks it)
  return 0;
}

int run_match_host(emqx_gm_ctx* ctx, const emqx_gm_index* idx, const uint8_t* tb, const uint64_t* to, uint64_t n,
                   uint32_t flags, emqx_gm_csr* out) {
  // the devices: this context, then the members the index has replicas on
  std::vector<emqx_gm_ctx*> mem{ctx};
  std::vector<const emqx_gm_index*> rix{idx};
  for (size_t k = 0; k < ctx->members.size() && k < idx->reps.size(); ++k) {
    mem.push_back(ctx->members[k]);
    rix.push_back(idx->reps[k]);
  }
  const uint64_t K = mem.size();
  // chunks: ~6 per device and call (so PCIe in, the kernels and PCIe out
  // overlap) of 256K..4M topics, at most 512 MiB of text; GM_HOST_CHUNK pins
  // the size (tests)
  const uint64_t CH = std::max<uint64_t>(
      1024, env_u64("GM_HOST_CHUNK", std::min<uint64_t>(4u << 20, std::max<uint64_t>(256u << 10, n / (6 * K)))));
  const uint64_t CB = 512ull << 20;
  std::vector<uint64_t> cb{0};
  while (cb.back() < n) {
    const uint64_t c0 = cb.back();
    uint64_t lo = c0 + 1, hi = std::min(n, c0 + CH);
    if (to[hi] < to[c0] || to[lo] < to[c0]) return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
    if (to[hi] - to[c0] > CB) {
      while (lo < hi) {  // largest c1 with the chunk's text <= CB
        const uint64_t mm = (lo + hi + 1) / 2;
        if (to[mm] >= to[c0] && to[mm] - to[c0] <= CB) lo = mm;
        else hi = mm - 1;
      }
      hi = lo;
    }
    if (to[hi] < to[c0] || to[hi] - to[c0] >= (1ull << 32))
      return set_err(ctx, EMQX_GM_EINVAL, "match: topic offsets not monotone");
    cb.push_back(hi);
  }
  const char* pe = knob("GM_HOST_PIPE");  // A/B: "serial" = the one-device serial path for every batch
  const bool serial = pe && !std::strcmp(pe, "serial") && K == 1;
  if (cb.size() <= 2 || serial) return run_host_serial(ctx, idx, tb, to, n, flags, out);
  return run_host_pipe(ctx, idx, tb, to, n, flags, mem, rix, cb, out);
}

}  // namespace gm

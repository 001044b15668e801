// gm_filters.h — the host table of an index snapshot's filters, in id order
// (ids are lexicographic ranks: Erlang binary order).
//
// An in-place update (gm_overlay.cpp, patch_update) must not copy the whole
// table per snapshot (C3: 10M filters, 250 MB of bytes): a table is an
// immutable, shared base (the filters of the last build or compaction) plus a
// small delta -- base positions deleted, filters inserted -- so deriving the
// next snapshot's table costs O(delta).  Once the delta passes 1/16 of the
// base the table is compacted (one O(n) copy, amortized over the updates that
// filled it).  Lookups are binary searches: at(rank) O(log n log d),
// rank_of(bytes) O(log n).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace gm {

inline int cmp_filter(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
  const int c = std::memcmp(a, b, std::min(la, lb));
  if (c) return c;
  return la < lb ? -1 : la > lb ? 1 : 0;
}

struct SortedFilters {  // sorted unique filters, packed
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};
  uint64_t n() const { return off.size() - 1; }
  const uint8_t* at(uint64_t i, uint64_t* len) const {
    *len = off[i + 1] - off[i];
    return bytes.data() + off[i];
  }
  // number of filters sorting strictly before f
  uint64_t lower_bound(const uint8_t* f, uint64_t len, bool* found) const {
    uint64_t lo = 0, hi = n();
    while (lo < hi) {
      const uint64_t m = (lo + hi) / 2;
      uint64_t l;
      const uint8_t* p = at(m, &l);
      if (cmp_filter(p, l, f, len) < 0) lo = m + 1;
      else hi = m;
    }
    *found = false;
    if (lo < n()) {
      uint64_t l;
      const uint8_t* p = at(lo, &l);
      *found = cmp_filter(p, l, f, len) == 0;
    }
    return lo;
  }
  void push(const uint8_t* p, uint64_t len) {
    bytes.insert(bytes.end(), p, p + len);
    off.push_back(bytes.size());
  }
};

class FilterTable {
 public:
  FilterTable() : base_(std::make_shared<SortedFilters>()) {}
  void set_base(std::shared_ptr<const SortedFilters> b) {
    base_ = std::move(b);
    tomb_.clear();
    ins_ = SortedFilters{};
    ipos_.clear();
  }
  uint64_t size() const { return base_->n() - tomb_.size() + ins_.n(); }
  uint64_t delta() const { return tomb_.size() + ins_.n(); }

  // the filter of id r
  const uint8_t* at(uint64_t r, uint64_t* len) const {
    if (tomb_.empty() && ipos_.empty()) return base_->at(r, len);
    // inserted filters with a rank below r, and whether r is one
    uint64_t lo = 0, hi = ipos_.size();
    while (lo < hi) {
      const uint64_t m = (lo + hi) / 2;
      if (ins_rank(m) < r) lo = m + 1;
      else hi = m;
    }
    if (lo < ipos_.size() && ins_rank(lo) == r) return ins_.at(lo, len);
    // else live base filter number r - lo: the smallest b with live(0..b) = r - lo + 1
    const uint64_t want = r - lo + 1;
    uint64_t a = 0, b = base_->n();
    while (a < b) {
      const uint64_t m = (a + b) / 2;
      if (m + 1 - tomb_le(m) < want) a = m + 1;
      else b = m;
    }
    return base_->at(a, len);
  }
  // number of filters sorting strictly before f; *found = f itself is in the table
  uint64_t rank_of(const uint8_t* f, uint64_t len, bool* found) const {
    bool fb;
    const uint64_t b = base_->lower_bound(f, len, &fb);
    if (tomb_.empty() && ipos_.empty()) {
      *found = fb;
      return b;
    }
    bool fi;
    const uint64_t k = ins_.lower_bound(f, len, &fi);
    *found = fi || (fb && !tombed(b));
    return b - tomb_lt(b) + k;
  }
  // every filter in id order: fn(id, bytes, len)
  template <class F> void for_each(F fn) const {
    uint64_t r = 0, t = 0, k = 0;
    const uint64_t nb = base_->n(), ni = ins_.n();
    for (uint64_t b = 0; b <= nb; ++b) {
      while (k < ni && ipos_[k] <= b) {
        uint64_t l;
        const uint8_t* p = ins_.at(k++, &l);
        fn(r++, p, l);
      }
      if (b == nb) break;
      if (t < tomb_.size() && tomb_[t] == b) {
        ++t;
        continue;
      }
      uint64_t l;
      const uint8_t* p = base_->at(b, &l);
      fn(r++, p, l);
    }
  }
  // The table after deleting the filters of ids `dels` (ascending) and
  // inserting `adds` (byte order, none present): O(delta) on a shared base,
  // compacted when the delta passes max(compact_min, base / 16).
  template <class StrSet>
  FilterTable apply(const std::vector<uint64_t>& dels, const StrSet& adds, uint64_t compact_min = 4096) const {
    FilterTable o;
    o.base_ = base_;
    // deletions: a base filter joins the tombstones, an inserted one leaves the inserts
    std::vector<uint8_t> drop_ins(ipos_.size(), 0);
    std::vector<uint32_t> nt;
    for (uint64_t r : dels) {
      uint64_t lo = 0, hi = ipos_.size();
      while (lo < hi) {
        const uint64_t m = (lo + hi) / 2;
        if (ins_rank(m) < r) lo = m + 1;
        else hi = m;
      }
      if (lo < ipos_.size() && ins_rank(lo) == r) {
        drop_ins[lo] = 1;
        continue;
      }
      const uint64_t want = r - lo + 1;
      uint64_t a = 0, b = base_->n();
      while (a < b) {
        const uint64_t m = (a + b) / 2;
        if (m + 1 - tomb_le(m) < want) a = m + 1;
        else b = m;
      }
      nt.push_back(uint32_t(a));
    }
    o.tomb_.resize(tomb_.size() + nt.size());
    std::merge(tomb_.begin(), tomb_.end(), nt.begin(), nt.end(), o.tomb_.begin());
    // inserts: the surviving old ones merged with the new, in byte order
    auto ai = adds.begin();
    auto put_add = [&]() {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(ai->data());
      bool f;
      o.ipos_.push_back(base_->lower_bound(p, ai->size(), &f));
      o.ins_.push(p, ai->size());
      ++ai;
    };
    for (uint64_t k = 0; k < ipos_.size(); ++k) {
      uint64_t l;
      const uint8_t* p = ins_.at(k, &l);
      while (ai != adds.end() &&
             cmp_filter(reinterpret_cast<const uint8_t*>(ai->data()), ai->size(), p, l) < 0)
        put_add();
      if (!drop_ins[k]) {
        o.ipos_.push_back(ipos_[k]);
        o.ins_.push(p, l);
      }
    }
    while (ai != adds.end()) put_add();
    if (o.delta() > std::max<uint64_t>(compact_min, base_->n() / 16)) o.compact();
    return o;
  }
  void compact() {
    auto b = std::make_shared<SortedFilters>();
    b->bytes.reserve(base_->bytes.size() + ins_.bytes.size());
    b->off.reserve(size() + 1);
    for_each([&](uint64_t, const uint8_t* p, uint64_t l) { b->push(p, l); });
    set_base(std::move(b));
  }

 private:
  std::shared_ptr<const SortedFilters> base_;
  std::vector<uint32_t> tomb_;  // base positions deleted, ascending
  SortedFilters ins_;           // inserted filters, byte order
  std::vector<uint64_t> ipos_;  // per inserted filter: base filters sorting before it

  uint64_t tomb_lt(uint64_t b) const { return std::lower_bound(tomb_.begin(), tomb_.end(), b) - tomb_.begin(); }
  uint64_t tomb_le(uint64_t b) const { return std::upper_bound(tomb_.begin(), tomb_.end(), b) - tomb_.begin(); }
  bool tombed(uint64_t b) const { return std::binary_search(tomb_.begin(), tomb_.end(), uint32_t(b)); }
  // the id of inserted filter k: the live base filters before it, plus the inserts before it
  uint64_t ins_rank(uint64_t k) const { return ipos_[k] - tomb_lt(ipos_[k]) + k; }
};

// The host side of an index's subscriber lists, per filter id: the offset of
// its segment in the subscriber CSR and its route mark (the filter is routed
// to another destination too: emqx_gm_index_update_subs ROUTE_ADD).  Like
// FilterTable, a shared immutable base plus a small delta, so a
// subscriber-only update (emqx_broker:subscribe/unsubscribe that add or drop
// no route, apps/emqx/src/emqx_broker.erl:147-165) derives the next
// snapshot's table in O(delta): the touched ids with their new counts (every
// offset past a touched id moves by the sum of the count changes before it)
// and the touched ids' marks.  Lookups are binary searches over the delta.
// Compacted (one O(n) pass) once the delta passes max(4096, n / 16).
class SubTable {
 public:
  SubTable() = default;
  // a materialized table: off[n + 1]; marks empty = a built index, where a
  // filter without subscribers is route-only
  SubTable(std::vector<uint64_t> off, std::vector<uint8_t> marks) {
    auto b = std::make_shared<Base>();
    b->off = std::move(off);
    b->pin = std::move(marks);
    base_ = std::move(b);
  }
  bool empty() const { return !base_ || base_->off.empty(); }  // no subscriber lists
  uint64_t n() const { return empty() ? 0 : base_->off.size() - 1; }
  uint64_t delta() const { return did_.size() + pover_.size(); }
  uint64_t off(uint64_t f) const {  // f in [0, n]
    const uint64_t k = uint64_t(std::lower_bound(did_.begin(), did_.end(), uint32_t(std::min<uint64_t>(f, ~0u))) -
                                did_.begin());
    return uint64_t(int64_t(base_->off[f]) + (k ? dcum_[k - 1] : 0));
  }
  uint64_t count(uint64_t f) const {
    auto it = std::lower_bound(did_.begin(), did_.end(), uint32_t(f));
    if (it != did_.end() && *it == f) return dnew_[it - did_.begin()];
    return base_->off[f + 1] - base_->off[f];
  }
  uint64_t total() const { return empty() ? 0 : off(n()); }
  bool pinned(uint64_t f) const {
    auto it = std::lower_bound(pover_.begin(), pover_.end(), std::make_pair(uint32_t(f), uint8_t(0)));
    if (it != pover_.end() && it->first == f) return it->second != 0;
    if (!base_->pin.empty()) return base_->pin[f] != 0;
    return base_->off[f + 1] == base_->off[f];
  }
  // the touched ids (ascending) and their running count changes: the device
  // derives the new offsets from these (new off[f] = old off[f] + the change
  // summed over touched ids below f)
  // The next snapshot's table, ids unchanged: `cnt` = (id, new count) for the
  // touched filters, `pin` = (id, mark) for the touched marks, both ascending.
  SubTable apply(const std::vector<std::pair<uint32_t, uint64_t>>& cnt,
                 const std::vector<std::pair<uint32_t, uint8_t>>& pin) const {
    SubTable o;
    o.base_ = base_;
    // counts: the old delta merged with the new (a new count replaces an old one)
    size_t a = 0, b = 0;
    while (a < did_.size() || b < cnt.size()) {
      uint32_t id;
      uint64_t c;
      if (b == cnt.size() || (a < did_.size() && did_[a] < cnt[b].first)) {
        id = did_[a], c = dnew_[a], ++a;
      } else {
        if (a < did_.size() && did_[a] == cnt[b].first) ++a;
        id = cnt[b].first, c = cnt[b].second, ++b;
      }
      const int64_t d = int64_t(c) - int64_t(base_->off[id + 1] - base_->off[id]);
      o.did_.push_back(id);
      o.dnew_.push_back(c);
      o.dcum_.push_back((o.dcum_.empty() ? 0 : o.dcum_.back()) + d);
    }
    a = b = 0;
    while (a < pover_.size() || b < pin.size()) {
      if (b == pin.size() || (a < pover_.size() && pover_[a].first < pin[b].first)) {
        o.pover_.push_back(pover_[a++]);
      } else {
        if (a < pover_.size() && pover_[a].first == pin[b].first) ++a;
        o.pover_.push_back(pin[b++]);
      }
    }
    if (o.delta() > std::max<uint64_t>(4096, n() / 16)) o.compact();
    return o;
  }
  const std::vector<uint32_t>& delta_ids() const { return did_; }
  const std::vector<int64_t>& delta_cum() const { return dcum_; }
  std::vector<uint64_t> offsets() const {  // materialized (index images)
    std::vector<uint64_t> r(n() + 1);
    for (uint64_t f = 0, k = 0; f <= n(); ++f) {
      while (k < did_.size() && did_[k] < f) ++k;
      r[f] = uint64_t(int64_t(base_->off[f]) + (k ? dcum_[k - 1] : 0));
    }
    return r;
  }
  std::vector<uint8_t> marks() const {
    std::vector<uint8_t> r(n());
    for (uint64_t f = 0; f < n(); ++f) r[f] = pinned(f) ? 1 : 0;
    return r;
  }
  void compact() { *this = SubTable(offsets(), marks()); }

 private:
  struct Base {
    std::vector<uint64_t> off;  // subscriber CSR offsets, n + 1
    std::vector<uint8_t> pin;   // route marks, n (empty: a count of 0 is the mark)
  };
  std::shared_ptr<const Base> base_;
  std::vector<uint32_t> did_;    // touched ids, ascending
  std::vector<uint64_t> dnew_;   // their counts
  std::vector<int64_t> dcum_;    // dcum_[k] = the count changes of did_[0..k] summed
  std::vector<std::pair<uint32_t, uint8_t>> pover_;  // touched marks, ascending
};

}  // namespace gm

// gm_overlay.cpp — incremental index maintenance.
//
// The reference mutates its trie in place inside mria transactions:
// emqx_router:do_add_route/2 -> emqx_router_utils:insert_trie_route/2 ->
// emqx_trie:insert/1, and do_delete_route/2 -> delete_trie_route ->
// emqx_trie:delete/1 (apps/emqx/src/emqx_router.erl:112-125, 164-172;
// emqx_router_utils.erl:33-70; emqx_trie.erl:107-136): insert is idempotent per
// topic key, delete only acts on a present key.  Here a device snapshot is
// immutable (readers may hold it, RCU): emqx_gm_index_update returns a NEW
// snapshot = the shared base snapshot minus tombstones plus a small delta
// index, and rebuilds a flat snapshot once the delta passes 1/8 of the base.
// Result rows use the ids of the updated set (lexicographic rank), exactly
// what a full rebuild would return.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <thread>

#include "gm_internal.h"

namespace gm {
namespace {

int cmp_bytes(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
  const int c = std::memcmp(a, b, std::min(la, lb));
  if (c) return c;
  return la < lb ? -1 : la > lb ? 1 : 0;
}

// Number of base filters sorting strictly before f; *found = exact hit.
uint64_t base_rank(const emqx_gm_index* base, const uint8_t* f, uint64_t len, bool* found) {
  return base->ft.rank_of(f, len, found);
}
const uint8_t* filter_at(const emqx_gm_index* idx, uint64_t id, uint64_t* len) { return idx->ft.at(id, len); }

// emqx_topic:wildcard/1 on the filter bytes
bool wildcard(const uint8_t* p, uint64_t len) {
  uint64_t ws = 0;
  for (uint64_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    if (i - ws == 1 && (p[ws] == '+' || p[ws] == '#')) return true;
    ws = i + 1;
  }
  return false;
}

// ---------------------------------------------------------------------------
// In-place update of a plain index: the new snapshot is a device copy of the
// previous one with the inserted filters' nodes, words and fields patched in
// and the deleted filters' fields cleared (worked out on the host mirror, the
// same bytes), then every filter id renumbered to the updated set's ranks by
// one device pass.  The result is an ordinary flat snapshot: a match on it
// costs exactly what a match on a rebuilt index costs (one pass, no overlay).
// ---------------------------------------------------------------------------
struct Words {  // '/'-separated words of one filter
  std::vector<std::pair<uint64_t, uint64_t>> w;  // (start, len)
  Words(const uint8_t* p, uint64_t len) {
    uint64_t ws = 0;
    for (uint64_t i = 0; i <= len; ++i)
      if (i == len || p[i] == '/') {
        w.emplace_back(ws, i - ws);
        ws = i + 1;
      }
  }
};
bool is1(const uint8_t* p, const std::pair<uint64_t, uint64_t>& w, char c) { return w.second == 1 && p[w.first] == c; }
// well formed for the in-place path: '#' only as the last word (anything else
// takes the overlay / rebuild path, which handles every byte string)
bool well_formed(const uint8_t* p, uint64_t len) {
  Words ws(p, len);
  for (size_t i = 0; i + 1 < ws.w.size(); ++i)
    if (is1(p, ws.w[i], '#')) return false;
  return true;
}

enum CurKind { CUR_ROOT, CUR_SLOT, CUR_INLINE };
struct Cur {
  CurKind kind = CUR_ROOT;
  uint32_t slot = 0;  // the node's slot, or for an inline node its parent's
  int table = 0;      // table of `slot`
  uint32_t v1 = 0;    // level-trie node
  uint32_t depth = 0;
  uint32_t pv1 = NONE, pwid = NONE;  // its parent and incoming word (for the parent's child refs)
  bool plus = false;                 // reached through '+'
};

struct NoRoom {};  // a table of the snapshot is full: the update rolls back and rebuilds

struct Patcher {
  Mirror& M;
  IndexView& v;  // the new snapshot's view (its host-side fields are patched here)
  // Blob ranges written (offset, bytes): uploaded over the device copy.  Writes
  // are field-granular on the id-bearing records (HotSlot, Node): the mirror's
  // filter-id fields are NOT renumbered after an update (only the device blob
  // is, by k_renumber), so a record's untouched id fields are stale on the host
  // and must not be uploaded.  A flag set on a field that also holds an id
  // (HOT_PLUS in hf / p_hf) goes to the device as an OR instead (orops).
  std::vector<std::pair<uint64_t, uint32_t>> dirty;
  std::vector<std::pair<uint64_t, uint32_t>> orops;  // (offset of a 32-bit word, bits to set)
  std::vector<std::pair<uint64_t, uint32_t>> undo_rng;  // every saved range, in order (rollback)
  uint32_t rh_clear = 0;                             // tables that took a key outside Robin Hood order
  uint64_t new_edges = 0;
  uint32_t max_depth = 0;
  // undo log: every write first saves the bytes it overwrites (rollback on NoRoom)
  std::vector<uint8_t> undo_bytes;
  uint64_t s_nodes_n, s_arena_n, s_dict_used, s_edge_used[EDGE_DEPTHS], s_hot_used[HOT_TABLES],
      s_mph_ovf_used[HOT_TABLES];

  Patcher(Mirror& m, IndexView& view) : M(m), v(view) {
    s_nodes_n = M.nodes_n;
    s_arena_n = M.arena_n;
    s_dict_used = M.dict_used;
    std::memcpy(s_edge_used, M.edge_used, sizeof(s_edge_used));
    std::memcpy(s_hot_used, M.hot_used, sizeof(s_hot_used));
    std::memcpy(s_mph_ovf_used, M.mph_ovf_used, sizeof(s_mph_ovf_used));
  }
  uint8_t* B() { return M.blob.data(); }
  Node* nodes() { return reinterpret_cast<Node*>(B() + M.o_nodes); }
  DictSlot* dict() { return reinterpret_cast<DictSlot*>(B() + M.o_dict); }
  EdgeSlot* edges() { return reinterpret_cast<EdgeSlot*>(B() + M.o_edges); }
  HotSlot* hot() { return reinterpret_cast<HotSlot*>(B() + M.o_hot); }
  uint8_t* arena() { return B() + M.o_arena; }
  uint32_t* efilt() { return reinterpret_cast<uint32_t*>(B() + M.o_efilt); }
  void save(uint64_t off, size_t n) {
    undo_rng.emplace_back(off, uint32_t(n));
    undo_bytes.insert(undo_bytes.end(), B() + off, B() + off + n);
  }
  // before writing n bytes at p
  void touch(const void* p, size_t n) {
    const uint64_t off = uint64_t(static_cast<const uint8_t*>(p) - B());
    dirty.emplace_back(off, uint32_t(n));
    save(off, n);
  }
  // set `bits` in a word whose other bits may be a (host-stale) filter id
  void orw(uint32_t& w, uint32_t bits) {
    if ((w & bits) == bits) return;
    const uint64_t off = uint64_t(reinterpret_cast<const uint8_t*>(&w) - B());
    save(off, 4);
    orops.emplace_back(off, bits);
    w |= bits;
  }
  // clear `bits` in such a word (an AND op on the device: offset | PATCH_AND)
  void andw(uint32_t& w, uint32_t bits) {
    if (!(w & bits)) return;
    const uint64_t off = uint64_t(reinterpret_cast<const uint8_t*>(&w) - B());
    save(off, 4);
    orops.emplace_back(off | PATCH_AND, bits);
    w &= ~bits;
  }
  template <class T> T& W(T& r) {
    touch(&r, sizeof(T));
    return r;
  }
  void rollback() {
    size_t q = undo_bytes.size();
    for (size_t k = undo_rng.size(); k-- > 0;) {
      q -= undo_rng[k].second;
      std::memcpy(B() + undo_rng[k].first, undo_bytes.data() + q, undo_rng[k].second);
    }
    M.nodes_n = s_nodes_n;
    M.arena_n = s_arena_n;
    M.dict_used = s_dict_used;
    std::memcpy(M.edge_used, s_edge_used, sizeof(s_edge_used));
    std::memcpy(M.hot_used, s_hot_used, sizeof(s_hot_used));
    std::memcpy(M.mph_ovf_used, s_mph_ovf_used, sizeof(s_mph_ovf_used));
  }

  // ---- word dictionary (dict_resolve's rules: length + head, tail against the arena)
  uint32_t dict_find(const uint8_t* w, uint64_t len) {
    const uint64_t head = word_head_host(w, len);
    for (uint64_t s = dict_slot(dict_hash_host(w, len), v.dict_mask);; s = (s + 1) & v.dict_mask) {
      const DictSlot& d = dict()[s];
      if (d.len == DICT_EMPTY_LEN) return NONE;
      if (d.len == len && d.head == head && (len <= 8 || std::memcmp(arena() + d.word + 8, w + 8, len - 8) == 0))
        return d.word;
    }
  }
  uint32_t word(const uint8_t* w, uint64_t len) {
    uint32_t id = dict_find(w, len);
    if (id != NONE) return id;
    const uint64_t own = len ? len : 1;  // every word owns >= 1 byte: ids stay unique
    if (M.arena_n + own > M.arena_cap || (M.dict_used + 1) * 2 > v.dict_mask + 1) throw NoRoom{};
    id = uint32_t(M.arena_n);
    touch(arena() + id, own);
    if (len) std::memcpy(arena() + id, w, len);
    else arena()[id] = 0;
    M.arena_n += own;
    uint64_t s = dict_slot(dict_hash_host(w, len), v.dict_mask);
    while (dict()[s].len != DICT_EMPTY_LEN) s = (s + 1) & v.dict_mask;
    W(dict()[s]) = DictSlot{word_head_host(w, len), uint32_t(len), id};
    ++M.dict_used;
    return id;
  }

  // ---- level trie (v1: slow path, literal lookups)
  uint32_t edge_get(uint32_t depth, uint32_t parent, uint32_t wid) {
    const int d = edge_depth(depth);
    EdgeSlot* tab = edges() + v.etab_off[d];
    const uint64_t key = edge_key(parent, wid), mask = v.etab_mask[d];
    for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
      if (tab[s].key == key) return tab[s].child;
      if (tab[s].key == EDGE_EMPTY) return NONE;
    }
  }
  void edge_put(uint32_t depth, uint32_t parent, uint32_t wid, uint32_t child) {
    const int d = edge_depth(depth);
    if ((M.edge_used[d] + 1) * 4 > (v.etab_mask[d] + 1) * 3) throw NoRoom{};  // load <= 0.75
    EdgeSlot* tab = edges() + v.etab_off[d];
    const uint64_t key = edge_key(parent, wid), mask = v.etab_mask[d];
    uint64_t s = edge_slot(key, mask);
    while (tab[s].key != EDGE_EMPTY) s = (s + 1) & mask;
    W(tab[s]) = EdgeSlot{key, child, 0};
    ++M.edge_used[d];
    ++new_edges;
  }
  uint32_t new_node() {
    if (M.nodes_n >= M.nodes_cap || M.nodes_n >= REF_X) throw NoRoom{};
    const uint32_t id = uint32_t(M.nodes_n++);
    W(nodes()[id]) = Node{NONE, NONE, NONE, 0};
    return id;
  }

  // ---- hot tables
  HotSlot* htab(int t) { return hot() + v.hot_off[t]; }
  uint64_t* mwords() { return reinterpret_cast<uint64_t*>(B() + M.o_mph); }
  uint32_t hot_find(int t, uint64_t key) { return hot_lookup_host(v, hot(), mwords(), t, key); }
  // Slots never move (a slot index is a hot id other keys hold), so the key
  // goes to the first empty slot from its home.  That keeps the table's Robin
  // Hood order (hot_resolve's early exit) as long as no resident on the way is
  // nearer its own home than the new key is at that slot; otherwise the
  // table's early exit is switched off (rh_clear).
  uint32_t hot_add(int t, uint64_t key) {
    const uint64_t cap = v.hot_cap[t];
    HotSlot* tab = htab(t);
    if (const uint32_t mc = v.mph_cap[t]) {
      // a perfect-hash table: the key's own slot when it is free, else the
      // overflow region (load <= 0.5; lookups probe it once its bit is set)
      uint64_t& bw = mwords()[v.mph_off[t] + mph_bucket(key, v.mph_nb[t])];
      W(bw) |= mph_bloom(key);  // the bucket's filter admits the new key (wherever it goes)
      uint64_t s = mph_slot(key, uint32_t(bw & 0xFFFFu), mc);
      if (tab[s].key != EDGE_EMPTY) {
        if (M.mph_ovf_used[t] + 1 > (cap - mc) / 2) throw NoRoom{};
        s = mph_ovf_home(key, mc, uint32_t(cap));
        while (tab[s].key != EDGE_EMPTY) s = s + 1 == cap ? mc : s + 1;
        ++M.mph_ovf_used[t];
        v.mph_ovf |= 1u << t;
      }
      W(tab[s]) = HotSlot{key, 0, HF_NONE, NONE, 0, HF_NONE, NONE};
      ++M.hot_used[t];
      return uint32_t(s);
    }
    if (!cap || (M.hot_used[t] + 1) * 5 > cap * 3) throw NoRoom{};  // load <= 0.6
    const uint64_t home = hot_slot(key, cap);
    uint64_t s = home, dist = 0;
    bool rh_ok = true;
    while (tab[s].key != EDGE_EMPTY) {
      const uint64_t h2 = hot_slot(tab[s].key, cap);
      if ((s >= h2 ? s - h2 : s + cap - h2) < dist) rh_ok = false;
      s = s + 1 == cap ? 0 : s + 1;
      ++dist;
    }
    W(tab[s]) = HotSlot{key, 0, HF_NONE, NONE, 0, HF_NONE, NONE};
    ++M.hot_used[t];
    if (!rh_ok) rh_clear |= 1u << t;
    return uint32_t(s);
  }
  static uint32_t hid(const Cur& c) {
    return c.kind == CUR_ROOT ? 0u : c.kind == CUR_SLOT ? c.slot : (c.slot | HOT_INLINE);
  }
  // the node's record: root -> IndexView fields, slot node -> its slot, inline
  // node -> p_* of its parent's slot.  F() records a field before a write
  // (the root's fields live in the view: nothing to record).
  uint32_t& F(const Cur& c, uint32_t& f) {
    if (c.kind != CUR_ROOT) touch(&f, 4);
    return f;
  }
  uint32_t& f_sig(const Cur& c) {
    return c.kind == CUR_ROOT ? v.root_sig : c.kind == CUR_SLOT ? htab(c.table)[c.slot].sig : htab(c.table)[c.slot].p_sig;
  }
  uint32_t& f_hf(const Cur& c) {
    return c.kind == CUR_SLOT ? htab(c.table)[c.slot].hf : htab(c.table)[c.slot].p_hf;
  }
  uint32_t& f_end(const Cur& c) {
    return c.kind == CUR_SLOT ? htab(c.table)[c.slot].end_filter : htab(c.table)[c.slot].p_end;
  }
  void set_hf(const Cur& c, uint32_t id) {  // 'match_#' of the node (keeps its HOT_PLUS flag)
    if (c.kind == CUR_ROOT) {
      v.root_hash = id == HF_NONE ? NONE : id;
      return;
    }
    uint32_t& f = F(c, f_hf(c));
    f = (f & HF_FLAGS) | id;
  }
  // A chain node on the path of a filter this update writes goes back to a
  // plain node (gm_common.h): its signature again, its tail free for an
  // inline '+' record; the walk then probes c1 / c2 in the tables, where they
  // still are.  Chains are only built by a rebuild.
  void unchain(const Cur& c) {
    if (c.kind != CUR_SLOT) return;
    HotSlot& S = htab(c.table)[c.slot];
    if (!(S.hf & HOT_CHAIN)) return;
    W(S.sig) = sig_bit(S.sig);
    W(S.p_sig) = 0;
    W(S.p_end) = NONE;
    andw(S.hf, HOT_CHAIN);
  }
  // a node's first exact child: set NF_HAS_EXACT and the REF_X bit of the
  // references to it (its parent's edge, and plus_child when it is a '+' child)
  void gain_exact(const Cur& c) {
    if (nodes()[c.v1].flags & NF_HAS_EXACT) return;
    W(nodes()[c.v1].flags) |= NF_HAS_EXACT;
    if (c.pv1 == NONE) return;  // the root: no reference
    const int d = edge_depth(c.depth - 1);
    EdgeSlot* tab = edges() + v.etab_off[d];
    const uint64_t key = edge_key(c.pv1, c.pwid), mask = v.etab_mask[d];
    for (uint64_t s = edge_slot(key, mask);; s = (s + 1) & mask) {
      if (tab[s].key == key) {
        W(tab[s]).child |= REF_X;
        break;
      }
      if (tab[s].key == EDGE_EMPTY) break;
    }
    if (c.plus) W(nodes()[c.pv1].plus_child) |= REF_X;
  }

  // Insert a well-formed filter with (temporary) id fid.  Throws NoRoom.
  void insert(const uint8_t* p, uint64_t len, uint32_t fid, bool wild) {
    Words ws(p, len);
    Cur c;
    for (size_t i = 0; i < ws.w.size(); ++i) {
      const auto& w = ws.w[i];
      if (is1(p, w, '#')) {  // the last word: the parent's 'match_#' (no hot node)
        const uint32_t hw = word(p + w.first, 1);
        v.hash_word = hw;
        uint32_t ch = edge_get(c.depth, c.v1, hw);
        if (ch == NONE) {
          ch = new_node();
          edge_put(c.depth, c.v1, hw, ch);
        }
        Node& hn = nodes()[ch & REF_MASK];
        W(hn.end_filter) = fid;
        W(hn.flags) |= NF_END_WILD;
        W(nodes()[c.v1].hash_filter) = fid;
        set_hf(c, fid);
        max_depth = std::max<uint32_t>(max_depth, c.depth + 1);
        return;
      }
      const bool plus = is1(p, w, '+');
      const uint32_t wid = word(p + w.first, w.second);
      if (plus) v.plus_word = wid;
      uint32_t ch = edge_get(c.depth, c.v1, wid);
      if (ch == NONE) {
        ch = new_node();
        edge_put(c.depth, c.v1, wid, ch);
        if (plus) {
          Node& pn = nodes()[c.v1];
          W(pn.plus_child) = ch;
          W(pn.flags) |= NF_HAS_PLUS;
        } else {
          gain_exact(c);
        }
      }
      Cur n;
      n.v1 = ch & REF_MASK;
      n.depth = c.depth + 1;
      n.pv1 = c.v1;
      n.pwid = wid;
      n.plus = plus;
      if (plus && plus_inline(c.depth, c.kind == CUR_SLOT)) {  // the '+' child lives in its parent's slot
        HotSlot& P = htab(c.table)[c.slot];
        if (!(P.hf & HOT_PLUS)) {
          orw(P.hf, HOT_PLUS);
          W(P.p_sig) = 0;
          W(P.p_hf) = HF_NONE;
          W(P.p_end) = NONE;
        }
        n.kind = CUR_INLINE;
        n.slot = c.slot;
        n.table = c.table;
      } else {
        const int t = hot_table(c.depth + 1);
        const uint64_t key = hot_key(hid(c), wid, c.depth);
        uint32_t sl = hot_find(t, key);
        if (sl == NONE) sl = hot_add(t, key);
        if (plus) {  // the parent (root or inline) gains its '+' flag
          if (c.kind == CUR_ROOT) {
            v.root_flags |= HOT_PLUS;
          } else {
            orw(f_hf(c), HOT_PLUS);
          }
        } else {  // the parent's exact-child signature and the table's exact-edge filter
          F(c, f_sig(c)) |= sig_bit(wid);
          if (v.efilt_mask[t]) {
            const uint32_t fh = edge_filter_hash(key);
            W(efilt()[v.efilt_off[t] + edge_filter_word(fh, v.efilt_mask[t])]) |= edge_filter_bits(fh);
          }
        }
        n.kind = CUR_SLOT;
        n.slot = sl;
        n.table = t;
      }
      c = n;
      unchain(c);
    }
    if (c.kind != CUR_ROOT) F(c, f_end(c)) = fid | (wild ? END_WILD : 0u);
    Node& en = nodes()[c.v1];
    W(en.end_filter) = fid;
    if (wild) W(en.flags) |= NF_END_WILD;
    max_depth = std::max<uint32_t>(max_depth, c.depth);
  }

  // Clear an indexed filter's fields (its nodes stay: an empty node matches nothing).
  void erase(const uint8_t* p, uint64_t len) {
    Words ws(p, len);
    const bool wf = well_formed(p, len);
    Cur c;
    uint32_t v1 = 0;
    for (size_t i = 0; i < ws.w.size(); ++i) {
      const auto& w = ws.w[i];
      const uint32_t wid = dict_find(p + w.first, w.second);
      if (wid == NONE) return;  // not indexed
      const uint32_t ch = edge_get(uint32_t(i), v1, wid);
      if (ch == NONE) return;
      const bool last = i + 1 == ws.w.size();
      if (last && is1(p, w, '#')) {
        W(nodes()[v1].hash_filter) = NONE;
        W(nodes()[ch & REF_MASK].end_filter) = NONE;
        if (wf) set_hf(c, HF_NONE);
        return;
      }
      if (wf) {  // follow the hot path (ill-formed filters have no hot fields)
        const bool plus = is1(p, w, '+');
        Cur n;
        if (plus && plus_inline(uint32_t(i), c.kind == CUR_SLOT)) {
          n.kind = CUR_INLINE;
          n.slot = c.slot;
          n.table = c.table;
        } else {
          const int t = hot_table(i + 1);
          const uint32_t sl = hot_find(t, hot_key(hid(c), wid, uint32_t(i)));
          if (sl == NONE) return;
          n.kind = CUR_SLOT;
          n.slot = sl;
          n.table = t;
        }
        c = n;
        unchain(c);
      }
      v1 = ch & REF_MASK;
    }
    W(nodes()[v1].end_filter) = NONE;
    if (wf && c.kind != CUR_ROOT) F(c, f_end(c)) = NONE;
  }
};

// rmap[temporary id] -> final id (NONE: deleted) over every filter-id field
// (the host twin of gm_match.hip's k_renumber), split over a few threads
void renumber_host(Mirror& M, const IndexView& v, const std::vector<uint32_t>& rmap) {
  HotSlot* hot = reinterpret_cast<HotSlot*>(M.blob.data() + M.o_hot);
  Node* nd = reinterpret_cast<Node*>(M.blob.data() + M.o_nodes);
  uint64_t slots = 0;
  for (int t = 0; t < HOT_TABLES; ++t) slots = std::max(slots, v.hot_off[t] + v.hot_cap[t]);
  const uint32_t* r = rmap.data();
  const uint64_t n_nodes = M.nodes_n;
  auto work = [=](unsigned part, unsigned parts) {
    for (uint64_t s = slots * part / parts, e = slots * (part + 1) / parts; s < e; ++s) {
      HotSlot& h = hot[s];
      if (h.key == EDGE_EMPTY) continue;
      h.hf = renum_field(h.hf, HF_NONE, HF_FLAGS, r);
      h.end_filter = renum_field(h.end_filter, NONE, END_WILD, r);
      h.p_hf = renum_field(h.p_hf, HF_NONE, HF_FLAGS, r);
      h.p_end = renum_field(h.p_end, NONE, END_WILD, r);
    }
    for (uint64_t i = n_nodes * part / parts, e = n_nodes * (part + 1) / parts; i < e; ++i) {
      nd[i].hash_filter = renum_field(nd[i].hash_filter, NONE, 0, r);
      nd[i].end_filter = renum_field(nd[i].end_filter, NONE, 0, r);
    }
  };
  const unsigned parts = (slots + n_nodes) < (1u << 18) ? 1u : std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned p = 1; p < parts; ++p) th.emplace_back(work, p, parts);
  work(0, parts);
  for (auto& t : th) t.join();
}

}  // namespace

bool well_formed_filter(const uint8_t* p, uint64_t len) { return well_formed(p, len); }
uint64_t filter_rank(const emqx_gm_index* idx, const uint8_t* f, uint64_t len, bool* found) {
  return base_rank(idx, f, len, found);
}

// Returns 1 (nothing changed) when the snapshot's tables lack room: the caller rebuilds.
int patch_update(emqx_gm_ctx* ctx, emqx_gm_index* prev, const std::set<uint32_t>& tomb,
                 const std::set<std::string>& dset, emqx_gm_index** out, std::vector<uint32_t>* rmap_out,
                 bool trie_only, std::vector<RepTarget>* reps) {
  if (const int rc = load_mirror_blob(ctx, prev)) return rc;  // (a lazy mirror: the first update loads it)
  Mirror& M = *prev->mirror;
  const uint64_t nb = prev->info.n_filters, K = dset.size();
  if (nb + K >= HF_NONE) return 1;  // temporary ids must stay below HF_NONE: the rebuild reports it
  const uint64_t nf_new = nb - tomb.size() + K;
  if (nf_new > M.flen_cap) return 1;  // the other tables are checked per insert (NoRoom)
  // GM_UPDATE_TIMING: phase times on stderr (diagnostics)
  const bool timing = knob("GM_UPDATE_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[gm_update] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  auto* idx = new emqx_gm_index;
  idx->device = prev->device;
  idx->info = prev->info;
  IndexView v = prev->view;  // the new view: patched here, rebased per device below
  Patcher P{M, v};
  // final ids (IdShift: prev id -> new id, temporaries nb + k -> new id) from
  // O(delta) lists, and the new snapshot's host filter table derived from
  // prev's (FilterTable::apply: shared base + delta, gm_filters.h)
  IdShift shift;
  shift.nb = nb;
  shift.dels.assign(tomb.begin(), tomb.end());
  shift.addpos.reserve(K);
  for (const std::string& d : dset) {
    bool found;
    shift.addpos.push_back(base_rank(prev, reinterpret_cast<const uint8_t*>(d.data()), d.size(), &found));
  }
  idx->ft = prev->ft.apply(shift.dels, dset);
  const bool host = prev->dev_base == nullptr;  // a host-only index (CPU test): the mirror is the index
  std::vector<uint32_t> rmap;  // materialized only where the host needs it (host-only index, update_subs)
  if (host || rmap_out) rmap = shift.table();
  phase("ids");
  // clear the deleted, insert the new (temporary ids nb + k), on the mirror
  uint64_t twild = 0, dwild = 0;
  for (uint32_t b : tomb) {
    uint64_t bl;
    const uint8_t* bp = filter_at(prev, b, &bl);
    twild += wildcard(bp, bl);
    P.erase(bp, bl);
  }
  try {
    uint32_t k = 0;
    for (const std::string& d : dset) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data());
      const bool wild = wildcard(p, d.size());
      dwild += wild;
      P.insert(p, d.size(), uint32_t(nb + k), wild);
      ++k;
    }
  } catch (const NoRoom&) {  // the mirror back to prev's bytes; the caller rebuilds
    P.rollback();
    delete idx;
    phase("no room");
    return 1;
  }
  if (v.root_hash != NONE) v.root_hash = shift.map(v.root_hash);
  v.rh_mask &= ~P.rh_clear;
  v.n_nodes = uint32_t(M.nodes_n);
  v.n_filters = uint32_t(nf_new);
  phase("patch");
  // filter lengths (stats only, emqx_gm_matched_filter_bytes): rewritten in
  // final ids when first asked for (sum_filter_lengths), not per update
  idx->flen_stale = true;
  const size_t blob_bytes = trie_only ? M.blob.size() : prev->dev_bytes;  // the mirror ends at the CSR
  idx->dev_bytes = blob_bytes;
  // device: copy the previous blob, apply the patched ranges (still in temporary
  // ids), renumber every filter-id field -- on the first device and, at the
  // same time, on every member replica (the same plan applied to its own copy
  // of prev's tables, which are byte-identical to prev's)
  const uint8_t* OB = host ? M.blob.data() : static_cast<const uint8_t*>(prev->dev_base);
  std::atomic<uint32_t> reused{0}, fresh{0};
  auto device_half = [&](emqx_gm_ctx* c, const emqx_gm_index* src, emqx_gm_index* dst) -> int {
    std::unique_lock<std::recursive_mutex> lk(c->mu, std::defer_lock);
    if (c->parent) lk.lock();  // (a member: small calls hold only its lock)
    GM_HIP(c, hipSetDevice(src->device));
    if ((dst->dev_base = take_spare_blob(src->device, blob_bytes))) {
      reused.fetch_add(1);
    } else {
      fresh.fetch_add(1);
      const hipError_t e = hipMalloc(&dst->dev_base, blob_bytes);
      if (e != hipSuccess) {
        dst->dev_base = nullptr;
        return set_err(c, EMQX_GM_ENOMEM, std::string("index_update: hipMalloc: ") + hipGetErrorString(e));
      }
    }
    dst->dev_bytes = blob_bytes;
    if (const int rc = apply_patch_device(c, dst->dev_base, src->dev_base, blob_bytes, P.dirty, M.blob.data(), v,
                                          M.o_hot, M.o_nodes, M.nodes_n, shift, P.orops))
      return rc;
    // the view's pointers follow the new blob
    IndexView w = v;
    uint8_t* NB = static_cast<uint8_t*>(dst->dev_base);
    auto rebase = [&](auto p) {
      return p ? reinterpret_cast<decltype(p)>(NB + (reinterpret_cast<const uint8_t*>(p) - OB)) : p;
    };
    w.nodes = rebase(w.nodes);
    w.dict = rebase(w.dict);
    w.d0_root = rebase(w.d0_root);
    w.edges = rebase(w.edges);
    w.hot = rebase(w.hot);
    w.arena = rebase(w.arena);
    w.sub_off = trie_only ? nullptr : rebase(w.sub_off);  // trie_only: set by the caller
    w.sub_ids = trie_only ? nullptr : rebase(w.sub_ids);
    w.efilt = rebase(w.efilt);
    w.mph_word = rebase(w.mph_word);
    dst->dev_flen = reinterpret_cast<uint16_t*>(NB + M.o_flen);
    if (w.flags & IX_D0) {  // the root's '+' record again, from the patched and renumbered tables
      const int rc = refresh_d0(c, w, const_cast<uint32_t*>(w.d0_root));
      if (rc < 0) return rc;
      if (rc) w.flags &= ~IX_D0;
    }
    dst->view = w;
    return 0;
  };
  if (!host) {
    std::vector<RepTarget> none;
    std::vector<RepTarget>& R = reps ? *reps : none;
    for (auto& t : R) t.out = replica_shell(t.m, prev);
    const double t0 = now_ms();
    int rc = run_all(int(1 + R.size()), [&](int k) {
      return k == 0 ? device_half(ctx, prev, idx) : device_half(R[k - 1].m, R[k - 1].prev, R[k - 1].out);
    });
    hipSetDevice(prev->device);
    tl_ustats.device_ms = now_ms() - t0;
    tl_ustats.blobs_reused += reused.load();
    tl_ustats.blobs_fresh += fresh.load();
    phase("device");
    if (rc) {  // the mirror no longer matches any snapshot: later updates take the overlay path / rebuild
      for (auto& t : R) {
        free_index(t.out);
        t.out = nullptr;
      }
      free_index(idx);
      delete prev->mirror;
      prev->mirror = nullptr;
      return rc;
    }
    if (!R.empty()) {
      tl_ustats.replicas = uint32_t(R.size());
      tl_ustats.replica_mode = EMQX_GM_REP_PATCHED;
    }
  } else {
    // A host-only index (CPU tests) IS its mirror: renumber it.  A device index's
    // mirror keeps its filter-id fields stale: the patcher never reads them and
    // uploads only the fields it writes (Patcher::dirty / orops), so the host
    // side of an update stays O(delta) instead of a pass over the whole blob.
    renumber_host(M, v, rmap);
    idx->view = v;  // (a host-only index keeps the mirror's pointers)
    phase("renumber");
  }
  emqx_gm_index_info_t& in = idx->info;
  in.n_filters = nf_new;
  in.n_wildcard = prev->info.n_wildcard - twild + dwild;
  in.trie_empty = in.n_wildcard == 0;
  in.n_nodes = M.nodes_n;
  in.n_edges = prev->info.n_edges + P.new_edges;
  in.n_words = M.dict_used;
  in.max_depth = std::max(prev->info.max_depth, P.max_depth);
  in.device_bytes = blob_bytes;
  idx->level_nodes = prev->level_nodes ? prev->level_nodes + (M.nodes_n - P.s_nodes_n) : 0;  // new nodes, any depth
  if (rmap_out) *rmap_out = std::move(rmap);
  idx->mirror = prev->mirror;  // the mirror follows the newest snapshot
  prev->mirror = nullptr;
  if (reps && !host)
    for (auto& t : *reps) {  // the replicas' host side: the new snapshot's (shared bases)
      t.out->ft = idx->ft;
      t.out->info = idx->info;
      t.out->level_nodes = idx->level_nodes;
      t.out->flen_stale = true;
    }
  tl_ustats.kind = EMQX_GM_UPD_PATCH;
  *out = idx;
  return EMQX_GM_OK;
}

int update_index(emqx_gm_ctx* ctx, emqx_gm_index* prev, const uint8_t* fb, const uint64_t* fo, const uint8_t* ops,
                 uint64_t n_ops, emqx_gm_index** out) {
  if (!prev || !out) return set_err(ctx, EMQX_GM_EINVAL, "index_update: NULL argument");
  if (n_ops && (!fb || !fo || !ops)) return set_err(ctx, EMQX_GM_EINVAL, "index_update: NULL op buffers");
  if (!prev->gmap.empty()) return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update: shard index");
  emqx_gm_index* base = prev->ov ? prev->ov->base : prev;
  if (!base->subs.empty())  // (its CSR may live outside the tables: emqx_gm_index_update_subs)
    return set_err(ctx, EMQX_GM_EUNSUPPORTED, "index_update: index with subscriber lists (use index_update_subs)");
  std::set<uint32_t> tomb;
  std::set<std::string> dset;
  if (prev->ov) {
    tomb.insert(prev->ov->tomb.begin(), prev->ov->tomb.end());
    for (size_t k = 0; k + 1 < prev->ov->doff.size(); ++k)
      dset.emplace(reinterpret_cast<const char*>(prev->ov->dbytes.data() + prev->ov->doff[k]),
                   prev->ov->doff[k + 1] - prev->ov->doff[k]);
  }
  for (uint64_t i = 0; i < n_ops; ++i) {
    if (fo[i + 1] < fo[i]) return set_err(ctx, EMQX_GM_EINVAL, "index_update: offsets not monotone");
    const uint8_t* f = fb + fo[i];
    const uint64_t len = fo[i + 1] - fo[i];
    bool found;
    const uint64_t b = base_rank(base, f, len, &found);
    if (ops[i]) {  // insert (idempotent)
      if (found) tomb.erase(uint32_t(b));
      else dset.emplace(reinterpret_cast<const char*>(f), len);
    } else {  // delete (only if present)
      if (found) tomb.insert(uint32_t(b));
      else dset.erase(std::string(reinterpret_cast<const char*>(f), len));
    }
  }
  const uint64_t nb = base->info.n_filters;
  if (tomb.empty() && dset.empty()) {
    base->refs.fetch_add(1);
    *out = base;
    tl_ustats.kind = EMQX_GM_UPD_NONE;
    return EMQX_GM_OK;
  }
  // a plain snapshot with its mirror: patched in place into a new flat snapshot
  // (GM_UPDATE_OVERLAY: the overlay form below instead, A/B and tests)
  // (a filter with '#' before its last word takes the overlay; no room left in
  // the snapshot's tables: a rebuild, which restores the headroom)
  bool no_room = false;
  std::unique_lock<std::mutex> mirror_lock(prev->mirror_mu);  // updates of one snapshot from several contexts
  if (!prev->ov && prev->mirror && !knob("GM_UPDATE_OVERLAY") &&
      tomb.size() + dset.size() <= std::max<uint64_t>(4096, nb / 8)) {
    bool wf = true;
    for (const std::string& d : dset) wf = wf && well_formed(reinterpret_cast<const uint8_t*>(d.data()), d.size());
    if (wf) {
      // a multi-device context: every member patches its replica at once
      std::vector<RepTarget> reps = rep_targets(ctx, prev);
      const int rc = patch_update(ctx, prev, tomb, dset, out, nullptr, false, &reps);
      if (rc < 0) return rc;
      if (rc == 0) {
        const int ra = attach_replicas(*out, reps, 0);
        if (ra) {
          free_index(*out);
          *out = nullptr;
        }
        return ra;
      }
      no_room = true;
    }
  }
  mirror_lock.unlock();
  if (no_room || tomb.size() + dset.size() > std::max<uint64_t>(4096, nb / 8) || !base->dev_base) {
    // compaction: a flat snapshot of the updated set
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs{0};
    auto dit = dset.begin();
    auto tit = tomb.begin();
    base->ft.for_each([&](uint64_t b, const uint8_t* bp, uint64_t bl) {
      while (dit != dset.end() && cmp_bytes(reinterpret_cast<const uint8_t*>(dit->data()), dit->size(), bp, bl) < 0) {
        bytes.insert(bytes.end(), dit->begin(), dit->end());
        offs.push_back(bytes.size());
        ++dit;
      }
      if (tit != tomb.end() && *tit == b) {
        ++tit;
        return;
      }
      bytes.insert(bytes.end(), bp, bp + bl);
      offs.push_back(bytes.size());
    });
    for (; dit != dset.end(); ++dit) {
      bytes.insert(bytes.end(), dit->begin(), dit->end());
      offs.push_back(bytes.size());
    }
    bytes.resize(bytes.size() + 64, 0);
    const int rc = build_index(ctx, bytes.data(), offs.data(), offs.size() - 1, nullptr, nullptr, nullptr, out);
    tl_ustats.kind = EMQX_GM_UPD_REBUILD;
    return rc;
  }
  auto* idx = new emqx_gm_index;
  idx->device = base->device;
  auto* ov = new OverlayState;
  idx->ov = ov;
  base->refs.fetch_add(1);
  ov->base = base;
  ov->tomb.assign(tomb.begin(), tomb.end());
  ov->doff.push_back(0);
  uint64_t dwild = 0;
  for (const std::string& d : dset) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data());
    bool found;
    const uint32_t ip = uint32_t(base_rank(base, p, d.size(), &found));
    const uint32_t k = uint32_t(ov->ins.size());
    const uint32_t dead_below = uint32_t(std::lower_bound(ov->tomb.begin(), ov->tomb.end(), ip) - ov->tomb.begin());
    ov->ins.push_back(ip);
    ov->dgid.push_back(k + ip - dead_below);
    ov->dbytes.insert(ov->dbytes.end(), d.begin(), d.end());
    ov->doff.push_back(ov->dbytes.size());
    dwild += wildcard(p, d.size());
  }
  const uint64_t K = ov->ins.size();
  if (K) {
    std::vector<uint8_t> padded(ov->dbytes);
    padded.resize(padded.size() + 64, 0);
    const int rc = build_index(ctx, padded.data(), ov->doff.data(), K, nullptr, nullptr, nullptr, &ov->delta, nullptr,
                               ov->dgid.data());
    if (rc) {
      free_index(idx);
      return rc;
    }
  }
  // device: tombstone bitmap over base ids, its exclusive word prefix counts, insertion points
  const uint64_t words = nb / 32 + 1;
  std::vector<uint32_t> tbm(words, 0), tpre(words, 0);
  uint64_t twild = 0;
  for (uint32_t b : ov->tomb) {
    tbm[b >> 5] |= 1u << (b & 31);
    uint64_t bl;
    const uint8_t* bp = filter_at(base, b, &bl);
    twild += wildcard(bp, bl);
  }
  for (uint64_t w = 1; w < words; ++w) tpre[w] = tpre[w - 1] + uint32_t(__builtin_popcount(tbm[w - 1]));
  const size_t bytes = (2 * words + K + 1) * 4;
  hipError_t e = hipMalloc(&ov->dev, bytes);
  uint32_t* D = static_cast<uint32_t*>(ov->dev);
  if (e == hipSuccess) e = hipMemcpy(D, tbm.data(), words * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(D + words, tpre.data(), words * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess && K) e = hipMemcpy(D + 2 * words, ov->ins.data(), K * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_index(idx);
    return set_err(ctx, EMQX_GM_ENOMEM, std::string("index_update: device tables: ") + hipGetErrorString(e));
  }
  ov->d_tbm = D;
  ov->d_tpre = D + words;
  ov->d_ins = D + 2 * words;
  emqx_gm_index_info_t& in = idx->info;
  in = base->info;
  in.n_filters = nb - ov->tomb.size() + K;
  in.n_wildcard = base->info.n_wildcard - twild + dwild;
  in.trie_empty = in.n_wildcard == 0;
  in.device_bytes = base->info.device_bytes + bytes;
  tl_ustats.kind = EMQX_GM_UPD_OVERLAY;
  if (ov->delta) {
    in.n_nodes += ov->delta->info.n_nodes;
    in.n_edges += ov->delta->info.n_edges;
    in.n_words += ov->delta->info.n_words;
    in.device_bytes += ov->delta->info.device_bytes;
    in.max_depth = std::max(in.max_depth, ov->delta->info.max_depth);
  }
  *out = idx;
  return EMQX_GM_OK;
}

// Bytes of final id `id`: a delta filter, or the surviving base filter b with
// b - tombstones_below(b) + delta_before(b) == id.
int overlay_filter(const emqx_gm_index* idx, uint32_t id, const uint8_t** bytes, uint64_t* len) {
  const OverlayState& ov = *idx->ov;
  if (id >= idx->info.n_filters) return EMQX_GM_EINVAL;
  auto dg = std::lower_bound(ov.dgid.begin(), ov.dgid.end(), id);
  if (dg != ov.dgid.end() && *dg == id) {
    const size_t k = size_t(dg - ov.dgid.begin());
    *bytes = ov.dbytes.data() + ov.doff[k];
    *len = ov.doff[k + 1] - ov.doff[k];
    return EMQX_GM_OK;
  }
  const emqx_gm_index* base = ov.base;
  auto final_id = [&](uint64_t b) -> uint64_t {
    const uint64_t dead = uint64_t(std::lower_bound(ov.tomb.begin(), ov.tomb.end(), uint32_t(b)) - ov.tomb.begin());
    const uint64_t before = uint64_t(std::upper_bound(ov.ins.begin(), ov.ins.end(), uint32_t(b)) - ov.ins.begin());
    return b - dead + before;
  };
  uint64_t lo = 0, hi = base->info.n_filters;  // smallest live b with final_id(b) >= id
  while (lo < hi) {
    const uint64_t m = (lo + hi) / 2;
    if (final_id(m) < id) lo = m + 1;
    else hi = m;
  }
  while (lo < base->info.n_filters && std::binary_search(ov.tomb.begin(), ov.tomb.end(), uint32_t(lo))) ++lo;
  if (lo >= base->info.n_filters || final_id(lo) != id) return EMQX_GM_EINVAL;
  *bytes = filter_at(base, lo, len);
  return EMQX_GM_OK;
}

void free_overlay(emqx_gm_index* idx) {
  OverlayState* ov = idx->ov;
  idx->ov = nullptr;
  if (ov->dev) {
    (void)hipSetDevice(idx->device);
    (void)hipFree(ov->dev);
  }
  if (ov->delta && ov->delta->refs.fetch_sub(1) == 1) free_index(ov->delta);
  if (ov->base && ov->base->refs.fetch_sub(1) == 1) free_index(ov->base);
  delete ov;
}

}  // namespace gm

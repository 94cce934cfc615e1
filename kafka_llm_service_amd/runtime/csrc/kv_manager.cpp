// Native paged-KV block manager + page-granular prefix cache (radix tree of 16-token pages).
//
// This is the engine's single-writer KV bookkeeping core (SURVEY.md §2.8 "Paged KV manager", "Prefix cache"):
//   * a fixed pool of `num_blocks` KV pages (each page = `page` tokens of every layer's K and V),
//   * per-sequence block tables,
//   * a prefix tree whose nodes are FULL pages keyed by (parent node, the page's token ids). A new request walks the
//     tree with its prompt and re-uses every matching page (shared system prompt + the thread's own history), so only
//     the uncached tail is prefilled. Pages are registered as soon as a sequence has written them completely (during
//     chunked prefill and during decode), which is what turns agent iteration k+1 and turn t+1 of a thread into
//     prefix hits,
//   * LRU eviction of unreferenced leaf pages when the free list runs dry,
//   * contiguous page runs: free pages are an ordered set handed out next-fit, a sequence takes its pages in runs of
//     consecutive block ids (a prefill chunk at once, decode growth `run` pages at a time, the spare ones reserved
//     for it), so a thread's history is a few long runs of the pool instead of one page every 64 blocks — its K/V
//     pages for a layer are read as long sweeps (DRAM pages, TLB reach). Reserved pages are reclaimed whenever the
//     pool runs short.
//
// Reference counting: node->ref = number of live sequences whose block table contains the node's page. A block is
// on the free list iff it is neither owned by a live sequence (exclusively) nor held by a tree node. A node with
// ref == 0 and no children is an evictable leaf (kept in an LRU set).
//
// The reference service has no counterpart (its LLM is remote: /root/reference/src/llm/portkey.py:367-379); the
// history re-send it performs on every request (/root/reference/server.py:395-404) is what this cache absorbs.
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace kafka {

struct Node {
  int64_t id = 0;
  int block = -1;
  Node* parent = nullptr;
  std::vector<int32_t> tokens;                       // page tokens (page entries)
  std::unordered_map<uint64_t, std::vector<Node*>> children;  // hash(tokens) -> nodes (collision list)
  int64_t n_children = 0;
  int64_t ref = 0;
  uint64_t last_use = 0;
  bool in_lru = false;
};

struct Seq {
  std::vector<int32_t> tokens;  // all tokens known for the sequence (prompt + generated)
  std::vector<int> blocks;      // block table
  std::vector<int> reserve;     // pages taken for this sequence's growth, not in its table yet (ascending)
  std::vector<Node*> nodes;     // nodes[i] != nullptr iff blocks[i] is a tree page referenced by this seq
  int64_t n_cached = 0;         // tokens whose KV came from the prefix cache at admission
  int64_t n_registered_pages = 0;
};

static inline uint64_t hash_page(const int32_t* t, int n) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)t[i] + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 1099511628211ull;
  }
  return h;
}

class KVManager {
 public:
  KVManager(int num_blocks, int page, bool prefix_cache, int run = 1)
      : num_blocks_(num_blocks), page_(page), prefix_cache_(prefix_cache), run_(std::max(1, run)) {
    if (num_blocks <= 0 || page <= 0) throw std::invalid_argument("num_blocks and page must be positive");
    for (int b = 0; b < num_blocks; ++b) free_.insert(free_.end(), b);
    root_ = std::make_unique<Node>();
    root_->id = 0;
  }
  ~KVManager() { clear_tree(root_.get()); }

  int page() const { return page_; }
  int num_blocks() const { return num_blocks_; }
  int num_free() const { return (int)free_.size(); }
  int num_reserved() const { return (int)n_reserved_; }
  int run() const { return run_; }
  // unreferenced cached pages (whole ref==0 subtrees: a sequence holding a page holds its whole chain)
  int num_evictable() const { return (int)n_unref_; }
  int num_cached_pages() const { return (int)n_nodes_; }
  // blocks that can be obtained right now (free + evictable + other sequences' reserves)
  int available() const { return (int)free_.size() + (int)n_unref_ + (int)n_reserved_; }

  bool has_seq(int64_t sid) const { return seqs_.count(sid) != 0; }

  // Admit a sequence with its prompt tokens. Walks the prefix tree over full pages, but never matches the whole
  // prompt: at least one token is left to compute (its logits are needed). Returns the number of cached tokens.
  int64_t add_sequence(int64_t sid, py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks) {
    if (seqs_.count(sid)) throw std::runtime_error("sequence already exists: " + std::to_string(sid));
    auto s = std::make_unique<Seq>();
    const int32_t* t = toks.data();
    const int64_t n = toks.size();
    s->tokens.assign(t, t + n);
    int64_t matched = 0;
    if (prefix_cache_ && n > 1) {
      Node* cur = root_.get();
      const int64_t max_pages = (n - 1) / page_;
      ++clock_;
      for (int64_t p = 0; p < max_pages; ++p) {
        Node* nx = find_child(cur, t + p * page_);
        if (!nx) break;
        acquire(nx);
        s->blocks.push_back(nx->block);
        s->nodes.push_back(nx);
        cur = nx;
        matched += page_;
      }
      s->n_registered_pages = (int64_t)s->nodes.size();
    }
    s->n_cached = matched;
    hit_tokens_ += matched;
    query_tokens_ += n;
    seqs_[sid] = std::move(s);
    return matched;
  }

  // Number of additional blocks sequence `sid` needs to hold `total_len` tokens.
  int blocks_needed(int64_t sid, int64_t total_len) const {
    const Seq& s = *get(sid);
    const int64_t need = (total_len + page_ - 1) / page_;
    return (int)std::max<int64_t>(0, need - (int64_t)s.blocks.size());
  }

  // Grow the block table to cover `total_len` tokens, evicting cached pages if needed. All-or-nothing.
  bool ensure_capacity(int64_t sid, int64_t total_len) {
    Seq& s = *get(sid);
    const int need = blocks_needed(sid, total_len);
    if (need == 0) return true;
    if (need > available()) return false;
    int left = need;
    // own reserve first
    while (left > 0 && !s.reserve.empty()) {
      take_table(s, s.reserve.front());
      s.reserve.erase(s.reserve.begin());
      --n_reserved_;
      --left;
    }
    if (left == 0) return true;
    if ((int64_t)free_.size() + n_unref_ < left) reclaim_reserves();
    // one run of consecutive pages: the whole need (a prefill chunk), or `run` pages for decode growth with the
    // spare ones reserved for this sequence
    const int want = std::max(left, run_);
    std::vector<int> got;
    if (want > 1 && (int64_t)free_.size() >= want && pop_run(want, got)) {
      for (int i = 0; i < left; ++i) take_table(s, got[i]);
      for (size_t i = left; i < got.size(); ++i) s.reserve.push_back(got[i]);
      n_reserved_ += (int64_t)got.size() - left;
      return true;
    }
    for (int i = 0; i < left; ++i) take_table(s, pop_block());
    return true;
  }

  // Append generated/known tokens to the sequence's token list.
  void append_tokens(int64_t sid, py::array_t<int32_t, py::array::c_style | py::array::forcecast> toks) {
    Seq& s = *get(sid);
    s.tokens.insert(s.tokens.end(), toks.data(), toks.data() + toks.size());
  }
  void append_token(int64_t sid, int32_t tok) { get(sid)->tokens.push_back(tok); }

  // Register every full page whose KV has been written (the first `computed_len` tokens) in the prefix tree.
  // Pages identical to an existing node are de-duplicated: the sequence adopts the tree's block and frees its own.
  void commit(int64_t sid, int64_t computed_len) {
    if (!prefix_cache_) return;
    Seq& s = *get(sid);
    const int64_t full = std::min<int64_t>(computed_len, (int64_t)s.tokens.size()) / page_;
    Node* cur = s.n_registered_pages ? s.nodes[s.n_registered_pages - 1] : root_.get();
    for (int64_t p = s.n_registered_pages; p < full && p < (int64_t)s.blocks.size(); ++p) {
      const int32_t* t = s.tokens.data() + p * page_;
      Node* ex = find_child(cur, t);
      if (ex) {
        // adopt the existing page; our exclusively-owned copy goes back to the free list
        acquire(ex);
        push_block(s.blocks[p]);
        s.blocks[p] = ex->block;
        s.nodes[p] = ex;
        cur = ex;
      } else {
        Node* nd = new_node(cur, t, s.blocks[p]);
        nd->ref = 1;
        s.nodes[p] = nd;
        cur = nd;
      }
      s.n_registered_pages = p + 1;
    }
  }

  // Release a sequence. Tree pages stay cached (evictable once unreferenced); private pages return to the pool.
  void free_sequence(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    Seq& s = *it->second;
    ++clock_;
    for (size_t i = 0; i < s.blocks.size(); ++i) {
      if (s.nodes[i]) release(s.nodes[i]);
      else push_block(s.blocks[i]);
    }
    for (int b : s.reserve) push_block(b);
    n_reserved_ -= (int64_t)s.reserve.size();
    seqs_.erase(it);
  }

  // Drop a sequence's KV beyond `keep_len` tokens (used by preemption-by-recompute to keep nothing but cached pages).
  std::vector<int> block_table(int64_t sid) const { return get(sid)->blocks; }
  int64_t num_tokens(int64_t sid) const { return (int64_t)get(sid)->tokens.size(); }
  int64_t num_cached(int64_t sid) const { return get(sid)->n_cached; }
  std::vector<int32_t> tokens(int64_t sid) const { return get(sid)->tokens; }

  // Fill an int32 [B, stride] block-table matrix for `sids` (columns beyond a sequence's table are left untouched).
  // The matrix is sized per step to the pages the step's kernels can touch (model_runner: ceil(len / page) of the
  // longest row), so a table with pages reserved further ahead is truncated to `stride` columns.
  void fill_block_tables(const std::vector<int64_t>& sids,
                         py::array_t<int32_t, py::array::c_style> out) {
    auto buf = out.mutable_unchecked<2>();
    const int64_t stride = buf.shape(1);
    if ((int64_t)sids.size() > buf.shape(0)) throw std::runtime_error("block table buffer too small (rows)");
    for (size_t r = 0; r < sids.size(); ++r) {
      const Seq& s = *get(sids[r]);
      const int64_t n = std::min<int64_t>((int64_t)s.blocks.size(), stride);
      int32_t* row = buf.mutable_data(r, 0);
      std::memcpy(row, s.blocks.data(), n * sizeof(int32_t));
    }
  }

  // slot ids (block * page + offset) for token positions [start, end) of `sid`, written at out[offset ...]
  void fill_slots(int64_t sid, int64_t start, int64_t end, py::array_t<int64_t, py::array::c_style> out,
                  int64_t offset) {
    const Seq& s = *get(sid);
    int64_t* o = out.mutable_data();
    if (offset + (end - start) > out.size()) throw std::runtime_error("slot buffer too small");
    for (int64_t p = start; p < end; ++p) {
      const int64_t bi = p / page_;
      if (bi >= (int64_t)s.blocks.size()) throw std::runtime_error("slot beyond allocated blocks");
      o[offset + p - start] = (int64_t)s.blocks[bi] * page_ + (p % page_);
    }
  }

  // Number of leading block-table entries identical across all `sids` (the shared prefix in pages).
  int64_t common_prefix_blocks(const std::vector<int64_t>& sids) const {
    if (sids.empty()) return 0;
    const Seq& a = *get(sids[0]);
    int64_t n = (int64_t)a.blocks.size();
    for (size_t i = 1; i < sids.size() && n > 0; ++i) {
      const Seq& b = *get(sids[i]);
      int64_t m = std::min<int64_t>(n, (int64_t)b.blocks.size());
      int64_t k = 0;
      while (k < m && a.blocks[k] == b.blocks[k]) ++k;
      n = k;
    }
    return n;
  }

  py::dict stats() const {
    py::dict d;
    d["num_blocks"] = num_blocks_;
    d["free"] = (int)free_.size();
    d["reserved"] = n_reserved_;
    d["evictable"] = n_unref_;
    d["cached_pages"] = n_nodes_;
    d["sequences"] = (int64_t)seqs_.size();
    d["hit_tokens"] = hit_tokens_;
    d["query_tokens"] = query_tokens_;
    d["evictions"] = evictions_;
    return d;
  }

  // Drop every unreferenced cached page (e.g. between benchmark phases).
  int64_t evict_all() {
    int64_t n = 0;
    while (!lru_.empty()) {
      evict_one();
      ++n;
    }
    return n;
  }

  // Internal consistency check used by the property tests: every block is in exactly one place.
  bool check_invariants() const {
    std::vector<int> owner(num_blocks_, 0);
    for (int b : free_) owner[b]++;
    std::vector<const Node*> stack{root_.get()};
    std::unordered_map<const Node*, int64_t> refs;
    while (!stack.empty()) {
      const Node* n = stack.back();
      stack.pop_back();
      if (n != root_.get()) owner[n->block]++;
      for (auto& kv : n->children)
        for (Node* c : kv.second) stack.push_back(c);
    }
    int64_t reserved = 0;
    for (auto& kv : seqs_) {
      const Seq& s = *kv.second;
      for (int b : s.reserve) owner[b]++;
      reserved += (int64_t)s.reserve.size();
      for (size_t i = 0; i < s.blocks.size(); ++i) {
        if (s.nodes[i]) {
          refs[s.nodes[i]]++;
          if (s.nodes[i]->block != s.blocks[i]) return false;
        } else {
          owner[s.blocks[i]]++;
        }
      }
    }
    for (int b = 0; b < num_blocks_; ++b)
      if (owner[b] != 1) return false;
    if (reserved != n_reserved_) return false;
    int64_t unref = 0;
    // node refs must equal the number of sequences referencing them
    stack.push_back(root_.get());
    while (!stack.empty()) {
      const Node* n = stack.back();
      stack.pop_back();
      if (n != root_.get()) {
        auto it = refs.find(n);
        const int64_t r = it == refs.end() ? 0 : it->second;
        if (r != n->ref) return false;
        if (n->ref == 0) ++unref;
        const bool should_lru = n->ref == 0 && n->n_children == 0;
        if (should_lru != n->in_lru) return false;
      }
      for (auto& kv : n->children)
        for (Node* c : kv.second) stack.push_back(c);
    }
    return unref == n_unref_;
  }

 private:
  struct LruKey {
    uint64_t t;
    int64_t id;
    Node* n;
    bool operator<(const LruKey& o) const { return t != o.t ? t < o.t : id < o.id; }
  };

  Seq* get(int64_t sid) const {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence " + std::to_string(sid));
    return it->second.get();
  }

  Node* find_child(Node* parent, const int32_t* t) {
    auto it = parent->children.find(hash_page(t, page_));
    if (it == parent->children.end()) return nullptr;
    for (Node* c : it->second)
      if (std::memcmp(c->tokens.data(), t, page_ * sizeof(int32_t)) == 0) return c;
    return nullptr;
  }

  Node* new_node(Node* parent, const int32_t* t, int block) {
    Node* n = new Node();
    n->id = ++next_id_;
    n->block = block;
    n->parent = parent;
    n->tokens.assign(t, t + page_);
    n->last_use = ++clock_;
    parent->children[hash_page(t, page_)].push_back(n);
    if (parent->n_children++ == 0 && parent != root_.get()) lru_remove(parent);
    ++n_nodes_;
    return n;
  }

  void lru_insert(Node* n) {
    if (n->in_lru) return;
    lru_.insert(LruKey{n->last_use, n->id, n});
    n->in_lru = true;
  }
  void lru_remove(Node* n) {
    if (!n->in_lru) return;
    lru_.erase(LruKey{n->last_use, n->id, n});
    n->in_lru = false;
  }

  void acquire(Node* n) {
    if (n->ref++ == 0) {
      lru_remove(n);
      --n_unref_;
    }
    n->last_use = clock_;
  }
  void release(Node* n) {
    if (--n->ref == 0) {
      ++n_unref_;
      n->last_use = clock_;
      if (n->n_children == 0) lru_insert(n);
    }
  }

  void evict_one() {
    auto it = lru_.begin();
    Node* n = it->n;
    lru_.erase(it);
    n->in_lru = false;
    Node* p = n->parent;
    auto& bucket = p->children[hash_page(n->tokens.data(), page_)];
    bucket.erase(std::find(bucket.begin(), bucket.end(), n));
    if (bucket.empty()) p->children.erase(hash_page(n->tokens.data(), page_));
    free_.insert(n->block);
    delete n;
    --n_nodes_;
    --n_unref_;
    ++evictions_;
    if (--p->n_children == 0 && p != root_.get() && p->ref == 0) lru_insert(p);
  }

  void take_table(Seq& s, int b) {
    s.blocks.push_back(b);
    s.nodes.push_back(nullptr);
  }

  // next-fit: the first free page at or after the cursor (wrapping)
  int pop_block() {
    if (free_.empty()) {
      // idle speculative reserves go back before any cached prefix page is evicted (a reserve is only a guess at
      // a sequence's next pages; an evicted prefix page is a recompute for the next request that shares it)
      if (n_reserved_ > 0) reclaim_reserves();
      if (free_.empty()) {
        if (lru_.empty()) throw std::runtime_error("KV pool exhausted");
        evict_one();
      }
    }
    auto it = free_.lower_bound(cursor_);
    if (it == free_.end()) it = free_.begin();
    const int b = *it;
    free_.erase(it);
    cursor_ = b + 1;
    return b;
  }

  // n consecutive free pages at or after the cursor (a bounded search over candidate starts, wrapping once);
  // false (nothing taken) if no such run was found
  bool pop_run(int n, std::vector<int>& out) {
    out.clear();
    auto it = free_.lower_bound(cursor_);
    for (int pass = 0, tries = 0; pass < 2 && tries < 512; ++pass) {
      if (pass == 1) it = free_.begin();
      while (it != free_.end() && tries < 512) {
        ++tries;
        const int b0 = *it;
        auto jt = it;
        int k = 1;
        for (++jt; k < n && jt != free_.end() && *jt == b0 + k; ++jt) ++k;
        if (k == n) {
          for (int i = 0; i < n; ++i) out.push_back(b0 + i);
          free_.erase(it, jt);
          cursor_ = b0 + n;
          return true;
        }
        it = jt;  // the next candidate start: past the short run
      }
    }
    return false;
  }
  void push_block(int b) { free_.insert(b); }

  // every sequence's spare pages back to the pool (the pool ran short)
  void reclaim_reserves() {
    for (auto& kv : seqs_) {
      for (int b : kv.second->reserve) free_.insert(b);
      kv.second->reserve.clear();
    }
    n_reserved_ = 0;
  }

  void clear_tree(Node* n) {
    for (auto& kv : n->children)
      for (Node* c : kv.second) {
        clear_tree(c);
        delete c;
      }
    n->children.clear();
  }

  int num_blocks_;
  int page_;
  bool prefix_cache_;
  int run_;
  std::set<int> free_;
  int cursor_ = 0;
  int64_t n_reserved_ = 0;
  std::unique_ptr<Node> root_;
  std::set<LruKey> lru_;
  std::unordered_map<int64_t, std::unique_ptr<Seq>> seqs_;
  uint64_t clock_ = 0;
  int64_t next_id_ = 0;
  int64_t n_nodes_ = 0;
  int64_t n_unref_ = 0;
  int64_t hit_tokens_ = 0;
  int64_t query_tokens_ = 0;
  int64_t evictions_ = 0;
};

}  // namespace kafka

namespace kafka {
void register_plan_channel(py::module& m);  // plan_channel.cpp
void register_group_board(py::module& m);   // group_board.cpp
}

PYBIND11_MODULE(_kafka_runtime, m) {
  m.doc() = "kafka_llm_service_amd native runtime: paged KV block manager + prefix cache + TP plan channel";
  kafka::register_plan_channel(m);
  kafka::register_group_board(m);
  py::class_<kafka::KVManager>(m, "KVManager")
      .def(py::init<int, int, bool, int>(), py::arg("num_blocks"), py::arg("page") = 16,
           py::arg("prefix_cache") = true, py::arg("run") = 1)
      .def_property_readonly("run", &kafka::KVManager::run)
      .def("num_reserved", &kafka::KVManager::num_reserved)
      .def_property_readonly("page", &kafka::KVManager::page)
      .def_property_readonly("num_blocks", &kafka::KVManager::num_blocks)
      .def("num_free", &kafka::KVManager::num_free)
      .def("num_evictable", &kafka::KVManager::num_evictable)
      .def("num_cached_pages", &kafka::KVManager::num_cached_pages)
      .def("available", &kafka::KVManager::available)
      .def("has_seq", &kafka::KVManager::has_seq)
      .def("add_sequence", &kafka::KVManager::add_sequence)
      .def("blocks_needed", &kafka::KVManager::blocks_needed)
      .def("ensure_capacity", &kafka::KVManager::ensure_capacity)
      .def("append_tokens", &kafka::KVManager::append_tokens)
      .def("append_token", &kafka::KVManager::append_token)
      .def("commit", &kafka::KVManager::commit)
      .def("free_sequence", &kafka::KVManager::free_sequence)
      .def("block_table", &kafka::KVManager::block_table)
      .def("num_tokens", &kafka::KVManager::num_tokens)
      .def("num_cached", &kafka::KVManager::num_cached)
      .def("tokens", &kafka::KVManager::tokens)
      .def("fill_block_tables", &kafka::KVManager::fill_block_tables)
      .def("fill_slots", &kafka::KVManager::fill_slots)
      .def("common_prefix_blocks", &kafka::KVManager::common_prefix_blocks)
      .def("stats", &kafka::KVManager::stats)
      .def("evict_all", &kafka::KVManager::evict_all)
      .def("check_invariants", &kafka::KVManager::check_invariants);
}

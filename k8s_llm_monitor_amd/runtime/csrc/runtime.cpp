// Native serving runtime for k8s-llm-monitor-amd (host side, no HIP / torch dependency).
//
//  * BlockAllocator - paged KV-cache block free list (O(1) allocate/free, LIFO reuse so hot
//                     blocks stay resident in the MI355X L2/Infinity Cache).
//  * BPE            - byte-level BPE encoder: the same pre-tokenizer as engine/tokenizer.py's
//                     regex, merges applied by rank, per-word cache.  Prompts of a few thousand
//                     tokens encode in microseconds, keeping /api/v1/query admission off the GIL.
//  * pack_decode    - builds the decode-step staging arrays (ids, positions, slot mapping, lengths,
//                     block-table rows) for a batch in one call.
//  * StepChannel    - (step_channel.cpp) shared-memory ring carrying each step's inputs from the
//                     tensor-parallel leader to its workers.
//
// The reference has no native code; this replaces its Go process runtime pieces
// that matter for serving latency.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>
#include <list>

#include "runtime.h"

namespace py = pybind11;

namespace {

class BlockAllocator {
 public:
  explicit BlockAllocator(int num_blocks) : num_blocks_(num_blocks) {
    if (num_blocks < 0) throw std::invalid_argument("num_blocks < 0");
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
    used_.assign(num_blocks, 0);
  }
  std::optional<std::vector<int>> allocate(int n) {
    if (n < 0 || n > (int)free_.size()) return std::nullopt;
    std::vector<int> out(n);
    for (int i = 0; i < n; ++i) {
      out[i] = free_.back();
      free_.pop_back();
      used_[out[i]] = 1;
    }
    return out;
  }
  void free(const std::vector<int>& blocks) {
    for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) {
      const int b = *it;
      if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id out of range");
      if (!used_[b]) throw std::runtime_error("double free of KV block " + std::to_string(b));
      used_[b] = 0;
      free_.push_back(b);
    }
  }
  int num_free() const { return (int)free_.size(); }
  int num_blocks() const { return num_blocks_; }

 private:
  int num_blocks_;
  std::vector<int> free_;
  std::vector<uint8_t> used_;
};

// ---------------------------------------------------------------------------------------------
// BlockPool - reference-counted KV blocks with a prefix cache.  A full block of prompt tokens is
// identified by a chained hash (block_hashes: the hash of block i covers tokens [0, 16 (i+1))),
// so a lookup of a prompt's hash chain finds the longest already-computed prefix.  Blocks whose
// last reference is dropped stay cached (LRU) until a fresh allocation needs them.
inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

std::vector<uint64_t> block_hashes(const std::vector<int>& tokens, int block_size, uint64_t seed) {
  if (block_size <= 0) throw std::invalid_argument("block_size <= 0");
  std::vector<uint64_t> out;
  const size_t nfull = tokens.size() / (size_t)block_size;
  out.reserve(nfull);
  uint64_t h = splitmix64(seed ^ 0x6b38c1a7d2e5f091ull);
  for (size_t b = 0; b < nfull; ++b) {
    uint64_t x = h;
    for (int i = 0; i < block_size; ++i) x = splitmix64(x ^ (uint64_t)(uint32_t)tokens[b * block_size + i]);
    h = x ? x : 1;  // 0 is reserved for "no hash"
    out.push_back(h);
  }
  return out;
}

class BlockPool {
 public:
  explicit BlockPool(int num_blocks)
      : num_blocks_(num_blocks), ref_(num_blocks, 0), hash_(num_blocks, 0), in_lru_(num_blocks, 0),
        lru_pos_(num_blocks) {
    if (num_blocks < 0) throw std::invalid_argument("num_blocks < 0");
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }

  // Number of leading hashes that are cached (no references taken).
  int peek(const std::vector<uint64_t>& hashes) const {
    int n = 0;
    for (uint64_t h : hashes) {
      if (map_.find(h) == map_.end()) break;
      ++n;
    }
    return n;
  }

  // Of the leading cached hashes, how many map to blocks with no reference (parked in the LRU):
  // matching those takes them out of the free pool, so admission must count them as consumed.
  int peek_idle(const std::vector<uint64_t>& hashes) const {
    int n = 0;
    for (uint64_t h : hashes) {
      auto it = map_.find(h);
      if (it == map_.end()) break;
      if (ref_[it->second] == 0) ++n;
    }
    return n;
  }

  // Longest cached prefix; takes one reference on every returned block.
  std::vector<int> match(const std::vector<uint64_t>& hashes) {
    std::vector<int> out;
    ++queries_;
    for (uint64_t h : hashes) {
      auto it = map_.find(h);
      if (it == map_.end()) break;
      const int b = it->second;
      if (ref_[b] == 0 && in_lru_[b]) {
        lru_.erase(lru_pos_[b]);
        in_lru_[b] = 0;
      }
      ++ref_[b];
      out.push_back(b);
    }
    hit_blocks_ += out.size();
    return out;
  }

  // n fresh blocks (free list first, then the least recently used cached blocks).
  std::optional<std::vector<int>> allocate(int n) {
    if (n < 0 || n > (int)(free_.size() + lru_.size())) return std::nullopt;
    std::vector<int> out(n);
    for (int i = 0; i < n; ++i) {
      int b;
      if (!free_.empty()) {
        b = free_.back();
        free_.pop_back();
      } else {
        b = lru_.front();
        lru_.pop_front();
        in_lru_[b] = 0;
        map_.erase(hash_[b]);
        hash_[b] = 0;
        ++evictions_;
      }
      ref_[b] = 1;
      out[i] = b;
    }
    return out;
  }

  // Register a block whose contents are the prefix with this chained hash.  If another block
  // already holds it, this one stays anonymous.
  void publish(int b, uint64_t h) {
    check(b);
    if (h == 0 || hash_[b] != 0 || map_.count(h)) return;
    map_[h] = b;
    hash_[b] = h;
  }

  void release(const std::vector<int>& blocks) {
    for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) {
      const int b = *it;
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("double free of KV block " + std::to_string(b));
      if (--ref_[b] == 0) {
        if (hash_[b] != 0) {
          lru_.push_back(b);
          lru_pos_[b] = std::prev(lru_.end());
          in_lru_[b] = 1;
        } else {
          free_.push_back(b);
        }
      }
    }
  }

  int num_free() const { return (int)(free_.size() + lru_.size()); }
  int num_blocks() const { return num_blocks_; }
  int num_cached() const { return (int)map_.size(); }
  int refcount(int b) const { check(b); return ref_[b]; }
  py::dict stats() const {
    py::dict d;
    d["cached_blocks"] = (int)map_.size();
    d["evictable_blocks"] = (int)lru_.size();
    d["hit_blocks"] = hit_blocks_;
    d["queries"] = queries_;
    d["evictions"] = evictions_;
    return d;
  }

 private:
  void check(int b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id out of range");
  }
  int num_blocks_;
  std::vector<int> free_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<uint8_t> in_lru_;
  std::list<int> lru_;
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int> map_;
  int64_t hit_blocks_ = 0, queries_ = 0, evictions_ = 0;
};

// ---------------------------------------------------------------------------------------------
// UTF-8 helpers + Python-compatible character classes of the pre-tokenizer regex
//   's|'t|'re|'ve|'m|'ll|'d| ?[A-Za-z]+| ?[0-9]{1,3}| ?[^\sA-Za-z0-9]+|\s+(?!\S)|\s+
inline int cp_len(unsigned char c) {
  if (c < 0x80) return 1;
  if ((c >> 5) == 0x6) return 2;
  if ((c >> 4) == 0xE) return 3;
  if ((c >> 3) == 0x1E) return 4;
  return 1;  // invalid byte: treat as a single unit
}

inline uint32_t cp_at(const std::string& s, size_t i, int* len) {
  const unsigned char c = s[i];
  int n = cp_len(c);
  if (i + n > s.size()) n = 1;
  *len = n;
  if (n == 1) return c;
  uint32_t v = c & (0xFF >> (n + 1));
  for (int k = 1; k < n; ++k) v = (v << 6) | (s[i + k] & 0x3F);
  return v;
}

inline bool is_space(uint32_t c) {  // Python str.isspace()
  return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
inline bool is_alpha(uint32_t c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
inline bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }
inline bool is_other(uint32_t c) { return !is_space(c) && !is_alpha(c) && !is_digit(c); }

// returns the end (byte offset) of the pre-token starting at i
size_t next_token(const std::string& s, size_t i) {
  const size_t n = s.size();
  int l;
  const uint32_t c = cp_at(s, i, &l);
  if (c == '\'' && i + 1 < n) {
    const char a = s[i + 1];
    if (a == 's' || a == 't' || a == 'm' || a == 'd') return i + 2;
    if (i + 2 < n) {
      const char b = s[i + 2];
      if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return i + 3;
    }
  }
  // " ?[A-Za-z]+ | ?[0-9]{1,3}| ?[^\sA-Za-z0-9]+": an optional single U+0020 prefix
  size_t st = i;
  uint32_t d = c;
  if (c == ' ' && i + 1 < n) {
    int l2;
    d = cp_at(s, i + 1, &l2);
    st = i + 1;
  }
  if (!(c == ' ' && st == i)) {
    if (is_alpha(d)) {
      size_t k = st;
      while (k < n && is_alpha((unsigned char)s[k])) ++k;
      return k;
    }
    if (is_digit(d)) {
      size_t k = st;
      int cnt = 0;
      while (k < n && cnt < 3 && is_digit((unsigned char)s[k])) ++k, ++cnt;
      return k;
    }
    if (is_other(d)) {
      size_t k = st;
      while (k < n) {
        int l3;
        const uint32_t e = cp_at(s, k, &l3);
        if (!is_other(e)) break;
        k += l3;
      }
      return k;
    }
  }
  // whitespace run: \s+(?!\S) then \s+
  size_t k = i;
  size_t last_start = i;
  while (k < n) {
    int l3;
    const uint32_t e = cp_at(s, k, &l3);
    if (!is_space(e)) break;
    last_start = k;
    k += l3;
  }
  if (k == n) return k;          // run reaches the end
  if (last_start > i) return last_start;  // leave the last space to prefix the next word
  return k;                      // single space before a non-space: \s+ fallback
}

class BPE {
 public:
  BPE(const std::vector<int>& left, const std::vector<int>& right) {
    if (left.size() != right.size()) throw std::invalid_argument("merge lists differ in length");
    for (size_t r = 0; r < left.size(); ++r) ranks_.emplace(key(left[r], right[r]), (int)r);
  }

  std::vector<int> encode(const std::string& s) const {
    std::vector<int> out;
    out.reserve(s.size() / 3 + 8);
    size_t i = 0;
    while (i < s.size()) {
      const size_t e = next_token(s, i);
      const std::string w = s.substr(i, e - i);
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = cache_.find(w);
        if (it != cache_.end()) {
          out.insert(out.end(), it->second.begin(), it->second.end());
          i = e;
          continue;
        }
      }
      std::vector<int> ids = merge_word(w);
      out.insert(out.end(), ids.begin(), ids.end());
      {
        std::lock_guard<std::mutex> g(mu_);
        if (cache_.size() < 500000) cache_.emplace(w, std::move(ids));
      }
      i = e;
    }
    return out;
  }

  std::vector<std::vector<int>> pretokenize(const std::string& s) const {
    std::vector<std::vector<int>> out;
    size_t i = 0;
    while (i < s.size()) {
      const size_t e = next_token(s, i);
      out.push_back({(int)i, (int)e});
      i = e;
    }
    return out;
  }

  size_t num_merges() const { return ranks_.size(); }

 private:
  static uint64_t key(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

  std::vector<int> merge_word(const std::string& w) const {
    std::vector<int> ids(w.begin(), w.end());
    for (auto& v : ids) v &= 0xFF;
    while (ids.size() > 1) {
      int best = -1;
      size_t bi = 0;
      for (size_t i = 0; i + 1 < ids.size(); ++i) {
        auto it = ranks_.find(key(ids[i], ids[i + 1]));
        if (it != ranks_.end() && (best < 0 || it->second < best)) {
          best = it->second;
          bi = i;
        }
      }
      if (best < 0) break;
      ids[bi] = 256 + best;
      ids.erase(ids.begin() + bi + 1);
    }
    return ids;
  }

  std::unordered_map<uint64_t, int> ranks_;
  mutable std::unordered_map<std::string, std::vector<int>> cache_;
  mutable std::mutex mu_;
};

// Decode-step staging: fills the pinned host arrays for a batch of sequences in one call.
//   last_tokens[i], num_tokens[i], block tables (flattened with offsets)
void pack_decode(py::array_t<int32_t> ids, py::array_t<int32_t> pos, py::array_t<int32_t> slots,
                 py::array_t<int32_t> lens, py::array_t<int32_t> bt, const std::vector<int>& last_tokens,
                 const std::vector<int>& num_tokens, const std::vector<std::vector<int>>& tables, int padded_b,
                 int block_size) {
  const int n = (int)last_tokens.size();
  auto I = ids.mutable_unchecked<1>();
  auto P = pos.mutable_unchecked<1>();
  auto S = slots.mutable_unchecked<1>();
  auto L = lens.mutable_unchecked<1>();
  auto B = bt.mutable_unchecked<2>();
  if (padded_b > I.shape(0) || padded_b > B.shape(0)) throw std::out_of_range("batch exceeds staging buffers");
  const int W = (int)B.shape(1);
  for (int i = 0; i < padded_b; ++i) {
    for (int j = 0; j < W; ++j) B(i, j) = 0;
    if (i >= n) {
      I(i) = 0;
      P(i) = 0;
      S(i) = -1;
      L(i) = 0;
      continue;
    }
    const int p = num_tokens[i] - 1;
    const auto& t = tables[i];
    if ((int)t.size() > W || p / block_size >= (int)t.size()) throw std::out_of_range("block table too short");
    I(i) = last_tokens[i];
    P(i) = p;
    S(i) = t[p / block_size] * block_size + p % block_size;
    L(i) = p + 1;
    for (size_t j = 0; j < t.size(); ++j) B(i, j) = t[j];
  }
}

}  // namespace

PYBIND11_MODULE(_k8sllm_runtime, m) {
  m.doc() = "k8s-llm-monitor-amd native serving runtime";
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int>())
      .def("allocate", &BlockAllocator::allocate)
      .def("free", &BlockAllocator::free)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks);
  py::class_<BPE>(m, "BPE")
      .def(py::init<const std::vector<int>&, const std::vector<int>&>())
      .def("encode", &BPE::encode, py::call_guard<py::gil_scoped_release>())
      .def("pretokenize", &BPE::pretokenize)
      .def_property_readonly("num_merges", &BPE::num_merges);
  m.def("pack_decode", &pack_decode);
  py::class_<BlockPool>(m, "BlockPool")
      .def(py::init<int>())
      .def("peek", &BlockPool::peek)
      .def("peek_idle", &BlockPool::peek_idle)
      .def("match", &BlockPool::match)
      .def("allocate", &BlockPool::allocate)
      .def("publish", &BlockPool::publish)
      .def("release", &BlockPool::release)
      .def("refcount", &BlockPool::refcount)
      .def("stats", &BlockPool::stats)
      .def_property_readonly("num_free", &BlockPool::num_free)
      .def_property_readonly("num_blocks", &BlockPool::num_blocks)
      .def_property_readonly("num_cached", &BlockPool::num_cached);
  m.def("block_hashes", &block_hashes, py::arg("tokens"), py::arg("block_size") = 16, py::arg("seed") = 0);
  register_step_channel(m);
}

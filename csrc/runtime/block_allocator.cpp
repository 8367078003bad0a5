// Native paged-KV block allocator with hash-chained prefix caching.
//
// Same semantics as engine/block_manager.py::BlockAllocator (the scheduler calls it
// for every sequence on every step, so it lives in C++):
//   * allocate(): a never-used / uncached free block first, else evict the LRU
//     cached free block (dropping its hash);
//   * free_block(): refcount--, a hashed block with refcount 0 stays addressable in
//     the LRU "cached free" list until reused;
//   * match_prefix(tokens): longest run of full blocks whose chained hashes are
//     cached (never the whole prompt: its last token must be recomputed);
//   * register(block, parent, tokens): publish a filled block.
// chain_hash is the same 64-bit FNV-style chain as the Python implementation, so
// the two are interchangeable (tests compare them operation by operation).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <deque>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

static inline uint64_t chain_hash(uint64_t parent, const int64_t* toks, size_t n) {
  uint64_t h = 1469598103934665603ULL ^ parent;
  for (size_t i = 0; i < n; ++i) {
    h ^= (uint64_t)toks[i] + 0x9E3779B97F4A7C15ULL;
    h *= 1099511628211ULL;
  }
  return h;
}

struct NoFreeBlocks : std::runtime_error {
  NoFreeBlocks() : std::runtime_error("no free KV blocks") {}
};

class BlockAllocator {
 public:
  BlockAllocator(int num_blocks, int block_size, bool prefix_caching)
      : num_blocks_(num_blocks), block_size_(block_size), prefix_caching_(prefix_caching),
        ref_(num_blocks, 0), has_hash_(num_blocks, 0), hash_of_(num_blocks, 0),
        lru_pos_(num_blocks) {
    for (int i = 0; i < num_blocks; ++i) free_.push_back(i);
  }

  int num_free() const { return (int)(free_.size() + lru_.size()); }
  double usage() const { return 1.0 - (double)num_free() / (double)std::max(1, num_blocks_); }

  int allocate() {
    int b;
    if (!free_.empty()) {
      b = free_.front();
      free_.pop_front();
    } else if (!lru_.empty()) {
      b = lru_.front();
      lru_.pop_front();
      in_lru_.erase(b);
      auto it = hash_to_block_.find(hash_of_[b]);
      if (it != hash_to_block_.end() && it->second == b) hash_to_block_.erase(it);
      has_hash_[b] = 0;
    } else {
      throw NoFreeBlocks();
    }
    ref_[b] = 1;
    return b;
  }

  void free_block(int b) {
    check(b);
    if (--ref_[b] > 0) return;
    if (has_hash_[b] && prefix_caching_) {
      lru_.push_back(b);
      lru_pos_[b] = std::prev(lru_.end());
      in_lru_.insert({b, true});
    } else {
      has_hash_[b] = 0;
      free_.push_back(b);
    }
  }

  void free_all(const std::vector<int>& blocks) {
    for (auto it = blocks.rbegin(); it != blocks.rend(); ++it) free_block(*it);
  }

  std::pair<std::vector<int>, uint64_t> match_prefix(const std::vector<int64_t>& tokens) {
    std::vector<int> out;
    uint64_t parent = 0;
    if (!prefix_caching_) return {out, parent};
    const size_t bs = (size_t)block_size_;
    size_t nfull = tokens.size() / bs;
    if (nfull * bs == tokens.size() && nfull > 0) nfull -= 1;
    for (size_t i = 0; i < nfull; ++i) {
      const uint64_t h = chain_hash(parent, tokens.data() + i * bs, bs);
      ++queries_;
      auto it = hash_to_block_.find(h);
      if (it == hash_to_block_.end()) break;
      const int b = it->second;
      ++hits_;
      if (ref_[b] == 0) {
        auto lit = in_lru_.find(b);
        if (lit != in_lru_.end()) {
          lru_.erase(lru_pos_[b]);
          in_lru_.erase(lit);
        }
      }
      ref_[b] += 1;
      out.push_back(b);
      parent = h;
    }
    return {out, parent};
  }

  uint64_t register_block(int block, uint64_t parent, const std::vector<int64_t>& tokens) {
    check(block);
    const uint64_t h = chain_hash(parent, tokens.data(), tokens.size());
    if (prefix_caching_ && hash_to_block_.find(h) == hash_to_block_.end()) {
      hash_to_block_[h] = block;
      has_hash_[block] = 1;
      hash_of_[block] = h;
    }
    return h;
  }

  int ref(int b) const { return ref_.at(b); }
  long hits() const { return hits_; }
  long queries() const { return queries_; }
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  bool prefix_caching() const { return prefix_caching_; }

 private:
  void check(int b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id out of range");
  }
  int num_blocks_, block_size_;
  bool prefix_caching_;
  std::vector<int> ref_;
  std::vector<char> has_hash_;
  std::vector<uint64_t> hash_of_;
  std::deque<int> free_;
  std::list<int> lru_;
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<int, bool> in_lru_;
  std::unordered_map<uint64_t, int> hash_to_block_;
  long hits_ = 0, queries_ = 0;
};

// slot mapping for a contiguous token range of one sequence (model-runner hot path)
static std::pair<std::vector<int32_t>, std::vector<int32_t>> slots_for(const std::vector<int>& table, int start,
                                                                       int n, int block_size) {
  std::vector<int32_t> slots(n), pos(n);
  for (int i = 0; i < n; ++i) {
    const int p = start + i;
    const size_t bi = (size_t)(p / block_size);
    if (bi >= table.size()) throw std::out_of_range("position beyond block table");
    slots[i] = table[bi] * block_size + p % block_size;
    pos[i] = p;
  }
  return {slots, pos};
}

void register_block_allocator(py::module_& m) {
  py::register_exception<NoFreeBlocks>(m, "NoFreeBlocks", PyExc_RuntimeError);
  m.def("chain_hash", [](uint64_t parent, const std::vector<int64_t>& t) { return chain_hash(parent, t.data(), t.size()); });
  m.def("slots_for", &slots_for);
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int, bool>())
      .def("allocate", &BlockAllocator::allocate)
      .def("free_block", &BlockAllocator::free_block)
      .def("free_all", &BlockAllocator::free_all)
      .def("match_prefix", &BlockAllocator::match_prefix)
      .def("register", &BlockAllocator::register_block)
      .def("usage", &BlockAllocator::usage)
      .def("ref", &BlockAllocator::ref)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("hits", &BlockAllocator::hits)
      .def_property_readonly("queries", &BlockAllocator::queries)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size)
      .def_property_readonly("prefix_caching", &BlockAllocator::prefix_caching);
}

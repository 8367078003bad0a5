// Native byte-level BPE encoder (the prompt-tokenisation hot path of /agent_rag:
// ~4 KB of evidence JSON per request, on the critical path of every admission).
//
// Encodes exactly like HF `tokenizers` for the two pre-tokeniser families the
// framework loads:
//   * GPT2  : ByteLevel(use_regex=True)  -- the built-in runbook BPE
//             's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
//   * LLAMA3: Split(llama-3 regex) + ByteLevel(use_regex=False) -- Llama-3 checkpoints
//             (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|
//              ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
// The regexes are implemented as hand-written scanners over code points (no regex
// engine, no backtracking), added tokens are split out first (leftmost-longest, as HF
// does), each pre-token is mapped through the GPT-2 bytes->unicode table and merged by
// rank (leftmost lowest-rank pair first == HF's heap order), with `ignore_merges`
// (Llama-3) honoured.  Merged pre-tokens are memoised; batch encodes run on worker
// threads with the GIL released.  tests/test_native_runtime_cpu.py checks token-for-
// token equality against HF on the synthetic corpus, Unicode and adversarial strings.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "unicode_tables.h"

namespace py = pybind11;

namespace {

enum : uint8_t { kOther = 0, kLetter = 1, kNumber = 2, kSpace = 3 };

bool in_ranges(uint32_t cp, const uint32_t (*r)[2], int n) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < r[mid][0]) hi = mid - 1;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}

// Unicode White_Space property (what \s matches in the regex engines HF uses)
bool is_ws(uint32_t c) {
  return (c >= 0x9 && c <= 0xD) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F ||
         c == 0x3000;
}

uint8_t klass(uint32_t c) {
  if (c < 128) {
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return kLetter;
    if (c >= '0' && c <= '9') return kNumber;
    return is_ws(c) ? kSpace : kOther;
  }
  if (is_ws(c)) return kSpace;
  if (in_ranges(c, kLetterRanges, kLetterRangesN)) return kLetter;
  if (in_ranges(c, kNumberRanges, kNumberRangesN)) return kNumber;
  return kOther;
}

struct Cp {
  uint32_t cp;
  uint32_t off;  // byte offset in the UTF-8 text
  uint8_t cls;
};

void decode_utf8(const std::string& s, size_t b, size_t e, std::vector<Cp>& out) {
  out.clear();
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  size_t i = b;
  while (i < e) {
    uint32_t c = p[i];
    int len = 1;
    if (c >= 0xF0 && i + 3 < e) {
      c = ((c & 0x07) << 18) | ((p[i + 1] & 0x3F) << 12) | ((p[i + 2] & 0x3F) << 6) | (p[i + 3] & 0x3F);
      len = 4;
    } else if (c >= 0xE0 && i + 2 < e) {
      c = ((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F);
      len = 3;
    } else if (c >= 0xC0 && i + 1 < e) {
      c = ((c & 0x1F) << 6) | (p[i + 1] & 0x3F);
      len = 2;
    }
    out.push_back({c, (uint32_t)i, klass(c)});
    i += len;
  }
}

inline bool is_nl(uint32_t c) { return c == '\r' || c == '\n'; }
inline uint32_t lower_ascii(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// contraction at i ('s 't 'm 'd / 're 've 'll); returns length or 0
int contraction(const std::vector<Cp>& c, size_t i, bool ci) {
  const size_t n = c.size();
  if (c[i].cp != '\'' || i + 1 >= n) return 0;
  const uint32_t x = ci ? lower_ascii(c[i + 1].cp) : c[i + 1].cp;
  if (x == 's' || x == 't' || x == 'm' || x == 'd') return 2;
  if (i + 2 < n) {
    const uint32_t y = ci ? lower_ascii(c[i + 2].cp) : c[i + 2].cp;
    if ((x == 'r' && y == 'e') || (x == 'v' && y == 'e') || (x == 'l' && y == 'l')) return 3;
  }
  return 0;
}

size_t run_of(const std::vector<Cp>& c, size_t k, uint8_t cls) {
  while (k < c.size() && c[k].cls == cls) ++k;
  return k;
}

// \s+(?!\S) | \s+  starting at whitespace position i
size_t ws_rule(const std::vector<Cp>& c, size_t i) {
  const size_t e = run_of(c, i, kSpace);
  if (e == c.size()) return e;
  return (e - i >= 2) ? e - 1 : e;
}

// pre-token boundaries (code-point indices) of one text segment
void pretokenize(const std::vector<Cp>& c, bool llama3, std::vector<std::pair<size_t, size_t>>& out) {
  out.clear();
  const size_t n = c.size();
  size_t i = 0;
  while (i < n) {
    size_t e = 0;
    if (int L = contraction(c, i, llama3)) {
      e = i + L;
    } else if (!llama3) {
      const size_t k = (c[i].cp == ' ' && i + 1 < n) ? i + 1 : i;
      const uint8_t cl = c[k].cls;
      if (cl == kLetter || cl == kNumber || cl == kOther) e = run_of(c, k, cl);
      else e = ws_rule(c, i);
    } else {
      const uint8_t c0 = c[i].cls;
      if (c0 == kLetter) {
        e = run_of(c, i, kLetter);
      } else if (c0 != kNumber && !is_nl(c[i].cp) && i + 1 < n && c[i + 1].cls == kLetter) {
        e = run_of(c, i + 1, kLetter);
      } else if (c0 == kNumber) {
        e = std::min(run_of(c, i, kNumber), i + 3);
      } else {
        const size_t k = (c[i].cp == ' ' && i + 1 < n && c[i + 1].cls == kOther) ? i + 1 : i;
        if (c[k].cls == kOther) {
          e = run_of(c, k, kOther);
          while (e < n && is_nl(c[e].cp)) ++e;
        } else {  // whitespace at i
          const size_t we = run_of(c, i, kSpace);
          size_t last_nl = SIZE_MAX;
          for (size_t j = i; j < we; ++j)
            if (is_nl(c[j].cp)) last_nl = j;
          e = last_nl != SIZE_MAX ? last_nl + 1 : ws_rule(c, i);
        }
      }
    }
    out.emplace_back(i, e);
    i = e;
  }
}

struct Merge {
  int rank;
  int id;
};

class BpeTokenizer {
 public:
  BpeTokenizer(const std::unordered_map<std::string, int>& vocab,
               const std::vector<std::pair<std::string, std::string>>& merges,
               const std::vector<std::tuple<std::string, int, bool>>& added, const std::string& mode,
               bool ignore_merges)
      : llama3_(mode == "llama3"), ignore_merges_(ignore_merges) {
    if (mode != "gpt2" && mode != "llama3") throw std::invalid_argument("mode must be gpt2 or llama3");
    // GPT-2 bytes_to_unicode
    std::vector<int> bs;
    for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
    for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
    for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
    std::vector<int> cs(bs);
    int extra = 0;
    for (int b = 0; b < 256; ++b) {
      if (std::find(bs.begin(), bs.end(), b) == bs.end()) {
        bs.push_back(b);
        cs.push_back(256 + extra++);
      }
    }
    for (size_t i = 0; i < bs.size(); ++i) byte_str_[bs[i]] = utf8(cs[i]);
    vocab_ = vocab;
    for (int b = 0; b < 256; ++b) {
      auto it = vocab_.find(byte_str_[b]);
      byte_id_[b] = it == vocab_.end() ? -1 : it->second;
    }
    int rank = 0;
    for (const auto& m : merges) {
      auto a = vocab_.find(m.first), b = vocab_.find(m.second), ab = vocab_.find(m.first + m.second);
      if (a != vocab_.end() && b != vocab_.end() && ab != vocab_.end())
        merges_[key(a->second, b->second)] = Merge{rank, ab->second};
      ++rank;
    }
    for (const auto& t : added) {
      const std::string& content = std::get<0>(t);
      if (!content.empty()) {
        added_.push_back({content, std::get<1>(t)});
        added_first_[(unsigned char)content[0]] = true;
      }
    }
    // longest first so a scan picks the longest added token at a position
    std::sort(added_.begin(), added_.end(),
              [](const auto& x, const auto& y) { return x.first.size() > y.first.size(); });
  }

  std::vector<int> encode(const std::string& text) {
    std::vector<int> out;
    Local lc;
    {
      py::gil_scoped_release nogil;
      std::shared_lock<std::shared_mutex> rd(mu_);
      encode_into(text, out, lc);
    }
    merge_cache(lc);
    return out;
  }

  std::vector<std::vector<int>> encode_batch(const std::vector<std::string>& texts, int threads) {
    std::vector<std::vector<int>> out(texts.size());
    const int T = std::max(1, std::min<int>(threads, (int)texts.size()));
    std::vector<Local> locals(T);
    {
      py::gil_scoped_release nogil;
      // several Python threads may encode at once (server event loop + engine thread):
      // batches read the shared cache under a shared lock, merges take it exclusively
      std::shared_lock<std::shared_mutex> rd(mu_);
      if (T == 1) {
        for (size_t i = 0; i < texts.size(); ++i) encode_into(texts[i], out[i], locals[0]);
      } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t)
          pool.emplace_back([&, t] {
            for (size_t i = t; i < texts.size(); i += T) encode_into(texts[i], out[i], locals[t]);
          });
        for (auto& th : pool) th.join();
      }
    }
    for (auto& lc : locals) merge_cache(lc);
    return out;
  }

  size_t cache_size() {
    std::shared_lock<std::shared_mutex> rd(mu_);
    return cache_.size();
  }

 private:
  using Local = std::unordered_map<std::string, std::vector<int>>;

  static uint64_t key(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

  static std::string utf8(int cp) {
    std::string s;
    if (cp < 0x80) {
      s += (char)cp;
    } else if (cp < 0x800) {
      s += (char)(0xC0 | (cp >> 6));
      s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xE0 | (cp >> 12));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    }
    return s;
  }

  void merge_cache(Local& lc) {
    if (lc.empty()) return;
    py::gil_scoped_release nogil;  // a batch in another thread may hold the read lock
    std::unique_lock<std::shared_mutex> wr(mu_);
    if (cache_.size() > (1u << 20)) cache_.clear();
    for (auto& kv : lc) cache_.emplace(std::move(kv.first), std::move(kv.second));
  }

  // one pre-token (raw bytes [b, e) of text) -> ids appended to out
  void bpe_piece(const std::string& text, size_t b, size_t e, std::vector<int>& out, Local& lc) {
    const std::string raw = text.substr(b, e - b);
    auto it = cache_.find(raw);  // under mu_ (shared); merges happen after join, exclusively
    if (it != cache_.end()) {
      out.insert(out.end(), it->second.begin(), it->second.end());
      return;
    }
    auto lt = lc.find(raw);
    if (lt != lc.end()) {
      out.insert(out.end(), lt->second.begin(), lt->second.end());
      return;
    }
    std::vector<int> w;
    w.reserve(raw.size());
    if (ignore_merges_) {
      std::string mapped;
      for (unsigned char ch : raw) mapped += byte_str_[ch];
      auto v = vocab_.find(mapped);
      if (v != vocab_.end()) w.push_back(v->second);
    }
    if (w.empty()) {
      for (unsigned char ch : raw) w.push_back(byte_id_[ch]);
      while (w.size() > 1) {
        int best = INT32_MAX, bi = -1, bid = -1;
        for (size_t i = 0; i + 1 < w.size(); ++i) {
          auto m = merges_.find(key(w[i], w[i + 1]));
          if (m != merges_.end() && m->second.rank < best) {
            best = m->second.rank;
            bi = (int)i;
            bid = m->second.id;
          }
        }
        if (bi < 0) break;
        w[bi] = bid;
        w.erase(w.begin() + bi + 1);
      }
    }
    out.insert(out.end(), w.begin(), w.end());
    if (raw.size() <= 256) lc.emplace(raw, std::move(w));
  }

  void encode_segment(const std::string& text, size_t b, size_t e, std::vector<int>& out, Local& lc) {
    if (b >= e) return;
    thread_local std::vector<Cp> cps;
    thread_local std::vector<std::pair<size_t, size_t>> spans;
    decode_utf8(text, b, e, cps);
    pretokenize(cps, llama3_, spans);
    for (const auto& sp : spans) {
      const size_t bb = cps[sp.first].off;
      const size_t ee = sp.second < cps.size() ? cps[sp.second].off : e;
      bpe_piece(text, bb, ee, out, lc);
    }
  }

  void encode_into(const std::string& text, std::vector<int>& out, Local& lc) {
    out.clear();
    size_t seg = 0, i = 0;
    while (i < text.size()) {
      int hit = -1;
      size_t hl = 0;
      if (added_first_[(unsigned char)text[i]]) {
        for (const auto& a : added_) {
          if (a.first.size() <= text.size() - i && text.compare(i, a.first.size(), a.first) == 0) {
            hit = a.second;
            hl = a.first.size();
            break;
          }
        }
      }
      if (hit >= 0) {
        encode_segment(text, seg, i, out, lc);
        out.push_back(hit);
        i += hl;
        seg = i;
      } else {
        ++i;
      }
    }
    encode_segment(text, seg, text.size(), out, lc);
  }

  bool llama3_, ignore_merges_;
  std::string byte_str_[256];
  int byte_id_[256];
  std::unordered_map<std::string, int> vocab_;
  std::unordered_map<uint64_t, Merge> merges_;
  std::vector<std::pair<std::string, int>> added_;
  bool added_first_[256] = {};
  std::unordered_map<std::string, std::vector<int>> cache_;
  std::shared_mutex mu_;
};

}  // namespace

void register_bpe(py::module_& m) {
  py::class_<BpeTokenizer>(m, "BpeTokenizer")
      .def(py::init<const std::unordered_map<std::string, int>&,
                    const std::vector<std::pair<std::string, std::string>>&,
                    const std::vector<std::tuple<std::string, int, bool>>&, const std::string&, bool>(),
           py::arg("vocab"), py::arg("merges"), py::arg("added"), py::arg("mode"), py::arg("ignore_merges"))
      .def("encode", &BpeTokenizer::encode)
      .def("encode_batch", &BpeTokenizer::encode_batch, py::arg("texts"), py::arg("threads") = 4)
      .def_property_readonly("cache_size", &BpeTokenizer::cache_size);
}

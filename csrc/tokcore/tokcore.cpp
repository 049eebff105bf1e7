// Native BPE cores of the GGUF tokenizers (nats_llm_studio_amd/tokenizer/bpe.py): the merge loops that
// the Python reference runs per pre-tokenised piece, here in C++ with the GIL released, so a burst of
// chat_model requests tokenises in parallel on the handler threads instead of serialising ~2 ms of
// pure-Python merging per prompt behind the interpreter lock (round-3 service profile: tokenisation p50
// 2.0 ms, p99 6.2 ms per request). In the reference this work happens inside LM Studio
// (`/root/reference/nats_llm_studio.go:158-179` forwards the chat payload to it).
//
//   ByteLevel: GPT-2 byte-level BPE (Llama-3, Granite, Qwen2). A piece's UTF-8 bytes start as the
//              single-byte tokens; the adjacent pair with the lowest merge rank is merged (leftmost first
//              among equal pairs) until none applies -- identical to bpe.py ByteLevelBPE._bpe.
//   Spm:       SentencePiece BPE (Mixtral / Llama-2): symbols are the UTF-8 characters of the
//              "▁"-normalised text; the adjacent pair whose concatenation is the highest-scoring
//              vocabulary entry is merged first (leftmost on ties); unknown symbols fall back to <0xXX>
//              byte tokens -- identical to bpe.py SentencePieceBPE._encode_plain.
//
//   Pretok:    the regex pre-tokenisers of bpe.py (LLAMA3_PRETOK, QWEN2_PRETOK, GPT2_PRETOK) as hand-written
//              scanners over code points, with \p{L} / \p{N} / \s from tables generated out of the same
//              `regex` module (tools/gen_unicode_tables.py); leftmost-first alternation and the greedy /
//              backtracking outcome of each alternative are reproduced case by case (comments below), and
//              tests/test_tokenizer.py fuzzes them against the regex module. ByteLevel.encode_text runs the
//              pre-tokeniser and the merges of a whole text without the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

#include "unicode_tables.h"

namespace py = pybind11;

namespace {

bool in_ranges(const CpRange* r, int n, uint32_t cp) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < r[mid].lo) hi = mid - 1;
    else if (cp > r[mid].hi) lo = mid + 1;
    else return true;
  }
  return false;
}
bool is_L(uint32_t c) { return c < 0x80 ? ((c | 0x20) - 'a' < 26u) : in_ranges(kLetter, kLetter_N, c); }
bool is_N(uint32_t c) { return c < 0x80 ? (c - '0' < 10u) : in_ranges(kNumber, kNumber_N, c); }
bool is_S(uint32_t c) { return c < 0x80 ? (c == ' ' || (c >= 9 && c <= 13)) : in_ranges(kSpace, kSpace_N, c); }
bool is_rn(uint32_t c) { return c == '\r' || c == '\n'; }

// UTF-8 -> code points with the byte offset of each (invalid bytes pass through as themselves: Python strings
// given to encode_text are always valid UTF-8)
void decode_utf8(const std::string& s, std::vector<uint32_t>& cp, std::vector<uint32_t>& off) {
  cp.clear();
  off.clear();
  for (size_t i = 0; i < s.size();) {
    const uint8_t c = (uint8_t)s[i];
    uint32_t v = c;
    size_t len = 1;
    if (c >= 0xF0 && i + 3 < s.size() + 0) {
      len = 4;
      v = ((c & 7u) << 18) | (((uint8_t)s[i + 1] & 63u) << 12) | (((uint8_t)s[i + 2] & 63u) << 6) | ((uint8_t)s[i + 3] & 63u);
    } else if (c >= 0xE0 && i + 2 < s.size()) {
      len = 3;
      v = ((c & 15u) << 12) | (((uint8_t)s[i + 1] & 63u) << 6) | ((uint8_t)s[i + 2] & 63u);
    } else if (c >= 0xC0 && i + 1 < s.size()) {
      len = 2;
      v = ((c & 31u) << 6) | ((uint8_t)s[i + 1] & 63u);
    }
    cp.push_back(v);
    off.push_back((uint32_t)i);
    i += len;
  }
  off.push_back((uint32_t)s.size());
}

enum PreMode { PRE_LLAMA3 = 0, PRE_QWEN2 = 1, PRE_GPT2 = 2 };

// length (in code points) of the match at i, >= 1 (every code point matches some alternative)
size_t pretok_match(const std::vector<uint32_t>& c, size_t i, int mode) {
  const size_t n = c.size();
  auto at = [&](size_t k) -> uint32_t { return k < n ? c[k] : 0xFFFFFFFFu; };
  auto other = [&](size_t k) { return k < n && !is_S(c[k]) && !is_L(c[k]) && !is_N(c[k]); };
  // contractions: (?i:'s|'t|'re|'ve|'m|'ll|'d) (llama3 / qwen2; case folding: s <-> S <-> U+017F), or the
  // case-sensitive list (gpt2)
  if (c[i] == '\'') {
    const bool ci = mode != PRE_GPT2;
    auto eq = [&](size_t k, char lc) {
      const uint32_t v = at(k);
      if (v == (uint32_t)lc) return true;
      if (!ci) return false;
      return v == (uint32_t)(lc - 32) || (lc == 's' && v == 0x17F);
    };
    if (eq(i + 1, 's') || eq(i + 1, 't') || eq(i + 1, 'm') || eq(i + 1, 'd')) return 2;
    if (eq(i + 1, 'r') && eq(i + 2, 'e')) return 3;
    if (eq(i + 1, 'v') && eq(i + 2, 'e')) return 3;
    if (eq(i + 1, 'l') && eq(i + 2, 'l')) return 3;
  }
  if (mode == PRE_GPT2) {
    // ' ?\p{L}+', ' ?\p{N}+', ' ?[^\s\p{L}\p{N}]+': an optional space belongs to the run after it
    const size_t j = (c[i] == ' ' && i + 1 < n) ? i + 1 : i;
    for (int kind = 0; kind < 3; ++kind) {
      auto ok = [&](size_t k) {
        return k < n && (kind == 0 ? is_L(c[k]) : kind == 1 ? is_N(c[k]) : other(k));
      };
      size_t s0 = ok(j) ? j : (ok(i) ? i : n);
      if (s0 == n) continue;
      size_t e = s0;
      while (ok(e)) ++e;
      return e - i;
    }
  } else {
    // [^\r\n\p{L}\p{N}]?\p{L}+
    if (!is_rn(c[i]) && !is_L(c[i]) && !is_N(c[i]) && i + 1 < n && is_L(c[i + 1])) {
      size_t e = i + 1;
      while (e < n && is_L(c[e])) ++e;
      return e - i;
    }
    if (is_L(c[i])) {
      size_t e = i;
      while (e < n && is_L(c[e])) ++e;
      return e - i;
    }
    // \p{N}{1,3} (llama3) / \p{N} (qwen2)
    if (is_N(c[i])) {
      const size_t cap = mode == PRE_QWEN2 ? 1 : 3;
      size_t e = i;
      while (e < n && e - i < cap && is_N(c[e])) ++e;
      return e - i;
    }
    // ' ?[^\s\p{L}\p{N}]+[\r\n]*'
    {
      const size_t s0 = (c[i] == ' ' && other(i + 1)) ? i + 1 : (other(i) ? i : n);
      if (s0 != n) {
        size_t e = s0;
        while (other(e)) ++e;
        while (e < n && is_rn(c[e])) ++e;
        return e - i;
      }
    }
    // '\s*[\r\n]+': up to and including the LAST \r / \n of the whitespace run at i
    {
      size_t w = i, last = n;
      while (w < n && is_S(c[w])) {
        if (is_rn(c[w])) last = w;
        ++w;
      }
      if (last != n) return last + 1 - i;
    }
  }
  // '\s+(?!\S)' then '\s+': the whitespace run, minus its last character when a non-space follows it
  size_t w = i;
  while (w < n && is_S(c[w])) ++w;
  if (w > i) {
    if (w == n) return w - i;
    if (w - i >= 2) return w - 1 - i;
    return 1;                                   // '\s+' of a single space before a non-space
  }
  return 1;                                     // (unreachable: every code point is L, N, \s or other)
}

struct PairHash {
  size_t operator()(uint64_t k) const { return std::hash<uint64_t>()(k * 0x9E3779B97F4A7C15ull); }
};

class ByteLevel {
 public:
  // byte_ids[b]: token of the single byte b; merges[i] = (left id, right id, merged id), rank i
  ByteLevel(std::vector<int32_t> byte_ids, const std::vector<std::tuple<int32_t, int32_t, int32_t>>& merges)
      : byte_ids_(std::move(byte_ids)) {
    if (byte_ids_.size() != 256) throw std::invalid_argument("ByteLevel: 256 byte ids expected");
    rank_.reserve(merges.size() * 2);
    for (size_t i = 0; i < merges.size(); ++i) {
      const auto& m = merges[i];
      const uint64_t k = key(std::get<0>(m), std::get<1>(m));
      if (rank_.find(k) == rank_.end()) rank_.emplace(k, std::make_pair((int32_t)i, std::get<2>(m)));
    }
  }

  // the whole text: pre-tokenise (mode: PreMode) and merge every piece
  void encode_text(const std::string& text, int mode, std::vector<int32_t>& out) const {
    std::vector<uint32_t> cp, off;
    decode_utf8(text, cp, off);
    for (size_t i = 0; i < cp.size();) {
      const size_t len = pretok_match(cp, i, mode);
      encode_piece(text.data() + off[i], off[i + len] - off[i], out);
      i += len;
    }
  }

  void encode_piece(const char* s, size_t n, std::vector<int32_t>& out) const {
    if (n == 0) return;
    std::vector<int32_t> sym(n), prev(n), next(n);
    std::vector<char> alive(n, 1);
    for (size_t i = 0; i < n; ++i) {
      sym[i] = byte_ids_[(uint8_t)s[i]];
      prev[i] = (int32_t)i - 1;
      next[i] = i + 1 < n ? (int32_t)i + 1 : -1;
    }
    if (n == 1) {
      out.push_back(sym[0]);
      return;
    }
    // min-heap of (rank, left position, left symbol, right symbol): stale entries are skipped on pop
    struct Cand {
      int32_t rank, pos, a, b;
      bool operator>(const Cand& o) const { return rank != o.rank ? rank > o.rank : pos > o.pos; }
    };
    std::priority_queue<Cand, std::vector<Cand>, std::greater<Cand>> heap;
    auto push = [&](int32_t i) {
      const int32_t j = next[i];
      if (i < 0 || j < 0) return;
      auto it = rank_.find(key(sym[i], sym[j]));
      if (it != rank_.end()) heap.push(Cand{it->second.first, i, sym[i], sym[j]});
    };
    for (int32_t i = 0; i + 1 < (int32_t)n; ++i) push(i);
    while (!heap.empty()) {
      const Cand c = heap.top();
      heap.pop();
      const int32_t i = c.pos;
      if (!alive[i]) continue;
      const int32_t j = next[i];
      if (j < 0 || sym[i] != c.a || sym[j] != c.b) continue;
      sym[i] = rank_.find(key(c.a, c.b))->second.second;
      alive[j] = 0;
      next[i] = next[j];
      if (next[j] >= 0) prev[next[j]] = i;
      push(prev[i]);
      push(i);
    }
    for (int32_t i = 0; i >= 0; i = next[i]) out.push_back(sym[i]);
  }

 private:
  static uint64_t key(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }
  std::vector<int32_t> byte_ids_;
  std::unordered_map<uint64_t, std::pair<int32_t, int32_t>, PairHash> rank_;   // pair -> (rank, merged)
};

class Spm {
 public:
  // tokens: UTF-8 text of every vocabulary entry ("▁" kept); scores; byte_ids[b]: <0xXX> token (or -1)
  Spm(const std::vector<std::string>& tokens, const std::vector<float>& scores, std::vector<int32_t> byte_ids)
      : scores_(scores), byte_ids_(std::move(byte_ids)) {
    vocab_.reserve(tokens.size() * 2);
    for (size_t i = 0; i < tokens.size(); ++i) vocab_[tokens[i]] = (int32_t)i;   // last id wins, as the Python
    // reference's {t: i} map and llama.cpp's token_to_id do for duplicate strings
  }

  // text: already "▁"-normalised (and prefixed) UTF-8
  void encode_text(const std::string& text, std::vector<int32_t>& out) const {
    if (text.empty()) return;
    std::vector<std::string> sym;
    for (size_t i = 0; i < text.size();) {
      const uint8_t c = (uint8_t)text[i];
      const size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
      sym.emplace_back(text.substr(i, std::min(len, text.size() - i)));
      i += len;
    }
    const int32_t n = (int32_t)sym.size();
    std::vector<int32_t> prev(n), next(n);
    std::vector<char> alive(n, 1);
    for (int32_t i = 0; i < n; ++i) {
      prev[i] = i - 1;
      next[i] = i + 1 < n ? i + 1 : -1;
    }
    struct Cand {
      float score;
      int32_t pos;
      size_t la, lb;     // lengths of the two symbols when pushed (a cheap staleness check)
      bool operator<(const Cand& o) const { return score != o.score ? score < o.score : pos > o.pos; }
    };
    std::priority_queue<Cand> heap;
    std::vector<std::string> ref_a(n), ref_b(n);
    auto push = [&](int32_t i) {
      if (i < 0) return;
      const int32_t j = next[i];
      if (j < 0) return;
      auto it = vocab_.find(sym[i] + sym[j]);
      if (it != vocab_.end()) heap.push(Cand{scores_[it->second], i, sym[i].size(), sym[j].size()});
    };
    for (int32_t i = 0; i + 1 < n; ++i) push(i);
    while (!heap.empty()) {
      const Cand c = heap.top();
      heap.pop();
      const int32_t i = c.pos;
      if (!alive[i]) continue;
      const int32_t j = next[i];
      if (j < 0 || !alive[j] || sym[i].size() != c.la || sym[j].size() != c.lb) continue;
      // the pair may have changed with the same lengths: confirm it still forms a vocabulary entry of
      // this score (the Python reference compares the symbol strings)
      auto it = vocab_.find(sym[i] + sym[j]);
      if (it == vocab_.end() || scores_[it->second] != c.score) continue;
      sym[i] += sym[j];
      alive[j] = 0;
      next[i] = next[j];
      if (next[j] >= 0) prev[next[j]] = i;
      push(prev[i]);
      push(i);
    }
    for (int32_t i = 0; i >= 0 && i < n; i = next[i]) {
      if (!alive[i]) continue;
      auto it = vocab_.find(sym[i]);
      if (it != vocab_.end()) {
        out.push_back(it->second);
      } else {
        for (uint8_t b : sym[i]) out.push_back(byte_ids_[b] >= 0 ? byte_ids_[b] : 0);
      }
    }
  }

 private:
  std::unordered_map<std::string, int32_t> vocab_;
  std::vector<float> scores_;
  std::vector<int32_t> byte_ids_;
};

}  // namespace

PYBIND11_MODULE(_tokcore, m) {
  m.doc() = "native BPE merge loops of the GGUF tokenizers (GIL released)";
  py::class_<ByteLevel>(m, "ByteLevel")
      .def(py::init<std::vector<int32_t>, const std::vector<std::tuple<int32_t, int32_t, int32_t>>&>())
      // pieces: the pre-tokeniser's matches as UTF-8 bytes -> the ids of all pieces, in order
      .def("encode_pieces", [](const ByteLevel& b, const std::vector<std::string>& pieces) {
        std::vector<int32_t> out;
        {
          py::gil_scoped_release r;
          out.reserve(pieces.size() * 2);
          for (const auto& p : pieces) b.encode_piece(p.data(), p.size(), out);
        }
        return out;
      })
      // text (UTF-8) -> ids: the native pre-tokeniser (mode 0 llama3, 1 qwen2, 2 gpt2) + merges, GIL released
      .def("encode_text", [](const ByteLevel& b, const std::string& text, int mode) {
        std::vector<int32_t> out;
        {
          py::gil_scoped_release r;
          out.reserve(text.size() / 3 + 4);
          b.encode_text(text, mode, out);
        }
        return out;
      })
      .def("encode_piece", [](const ByteLevel& b, const py::bytes& piece) {
        std::string s = piece;
        std::vector<int32_t> out;
        b.encode_piece(s.data(), s.size(), out);
        return out;
      });
  // the pre-tokeniser alone (tests): text -> the matched pieces as UTF-8 byte strings
  m.def("pretokenize", [](const std::string& text, int mode) {
    std::vector<uint32_t> cp, off;
    decode_utf8(text, cp, off);
    std::vector<py::bytes> out;
    for (size_t i = 0; i < cp.size();) {
      const size_t len = pretok_match(cp, i, mode);
      out.emplace_back(text.substr(off[i], off[i + len] - off[i]));
      i += len;
    }
    return out;
  });
  py::class_<Spm>(m, "Spm")
      .def(py::init<const std::vector<std::string>&, const std::vector<float>&, std::vector<int32_t>>())
      .def("encode", [](const Spm& s, const std::string& text) {
        std::vector<int32_t> out;
        {
          py::gil_scoped_release r;
          s.encode_text(text, out);
        }
        return out;
      });
}

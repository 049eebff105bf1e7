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
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

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
      .def("encode_piece", [](const ByteLevel& b, const py::bytes& piece) {
        std::string s = piece;
        std::vector<int32_t> out;
        b.encode_piece(s.data(), s.size(), out);
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

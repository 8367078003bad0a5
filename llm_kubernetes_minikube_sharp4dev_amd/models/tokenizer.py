"""Tokenizers.

* A real checkpoint's ``tokenizer.json`` (HF ``tokenizers``) is used when a model
  directory is given.
* Otherwise a built-in **byte-level BPE** with Llama-3's pre-tokenizer (the same split
  regex, ``ignore_merges``) and a 32k vocabulary is used, so random-init benchmark runs
  see prompt lengths of a real subword tokenizer and streamed output decodes to text.
  It is trained on text DISJOINT from the benchmark's synthetic generator and lexicon
  (``rag/synthetic.py``): the Python standard library's sources (English prose in
  docstrings and comments, code) plus the Italian message catalogs installed on the
  build image.  On the synthetic runbook prompts it yields ~3.5 chars/token (bench.py
  reports ``chars_per_token``), i.e. no better compression than Llama-3's own tokenizer
  would give on that pseudo-Italian text.  Trained once; the JSON ships in-tree.

Special tokens follow the Llama-3 chat format (Ollama applies the model's template
to ``/api/generate`` prompts).
"""
from __future__ import annotations

import json
import os
import threading
from pathlib import Path
from typing import Iterable, Optional

SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
            "<|eot_id|>", "[CLS]", "[SEP]", "[PAD]", "[UNK]", "[MASK]"]
_CACHE = Path(__file__).resolve().parent / "data" / "bpe_builtin_llama3_32k.json"
_lock = threading.Lock()


def _prose(src: str) -> str:
    """Docstrings and comments of one Python source (``ast`` / ``tokenize`` parse it; nothing
    is executed): the English prose of the file without its identifiers and code."""
    import ast
    import io
    import tokenize

    out = []
    try:
        for node in ast.walk(ast.parse(src)):
            if isinstance(node, (ast.Module, ast.ClassDef, ast.FunctionDef, ast.AsyncFunctionDef)):
                d = ast.get_docstring(node)
                if d:
                    out.append(d)
        for t in tokenize.generate_tokens(io.StringIO(src).readline):
            if t.type == tokenize.COMMENT and len(t.string) > 12:
                out.append(t.string.lstrip("#").strip())
    except (SyntaxError, ValueError, tokenize.TokenError, RecursionError):
        return ""
    return "\n".join(out)


def _training_text(max_chars: int = 12 << 20, code_share: float = 0.15):
    """Deterministic training stream with no synthetic-corpus text: the Italian strings of the
    ``.mo`` catalogs on the image (``gettext`` parses them; nothing executes), the English
    prose (docstrings, comments) of the Python standard library, and a slice of its code."""
    import glob
    import gettext
    import sysconfig

    it = []
    for pat in ("/usr/share/locale/it/**/*.mo", "/usr/share/locale-langpack/it/**/*.mo",
                "/opt/conda/**/it/LC_MESSAGES/*.mo", "/usr/local/lib/python3*/dist-packages/**/it/LC_MESSAGES/*.mo"):
        it += glob.glob(pat, recursive=True)
    ital = []
    for f in sorted(set(it)):
        try:
            with open(f, "rb") as fh:
                cat = gettext.GNUTranslations(fh)._catalog
        except Exception:
            continue
        ital += [v for _, v in sorted((str(k), v) for k, v in cat.items()) if isinstance(v, str) and v.strip()]
    std = Path(sysconfig.get_paths()["stdlib"])
    n = code = 0
    for i, f in enumerate(sorted(std.rglob("*.py"))):
        if "site-packages" in f.parts or "dist-packages" in f.parts:
            continue
        try:
            src = f.read_text(encoding="utf-8")
        except (OSError, UnicodeDecodeError):
            continue
        t = _prose(src)
        if code < code_share * max(n, 1):
            t += "\n" + src
            code += len(src)
        n += len(t)
        yield t
        if i % 64 == 0 and ital:  # the catalogs are small: interleave them throughout
            yield "\n".join(ital)
        if n >= max_chars:
            return


def _train_builtin(vocab_size: int = 32768):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE(ignore_merges=True))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=SPECIALS,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  show_progress=False)
    tok.train_from_iterator(_training_text(), trainer=trainer)
    return tok


LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                r"|\s*[\r\n]+|\s+(?!\S)|\s+")
_PROBES = ["Hello world's   test\n\n  x", "kubectl scale deploy/echoserver --replicas=3 -n dev",
           "\u00e8 perch\u00e9 \u4f60\u597d 12345 \U0001F600 <|eot_id|> 'Re 'LL x''y",
           '{"Question":"scala a 3","Evidence":[{"Id":"a.md#0","Score":0.71}]}\r\n\t end  ']


def native_encoder(hf_tok):
    """Native C++ BPE encoder (csrc/runtime/bpe.cpp) equivalent to ``hf_tok`` for the
    byte-level families it implements, or None (unsupported layout, runtime not built,
    or a probe mismatch)."""
    try:
        from ..native import runtime as nrt

        if not nrt.available():
            return None
        d = json.loads(hf_tok.to_str())
        m, pre = d.get("model") or {}, d.get("pre_tokenizer") or {}
        if (d.get("normalizer") is not None or m.get("type") != "BPE" or m.get("byte_fallback")
                or m.get("continuing_subword_prefix") or m.get("end_of_word_suffix") or m.get("dropout")):
            return None
        if pre.get("type") == "ByteLevel" and pre.get("use_regex", True) and not pre.get("add_prefix_space"):
            mode = "gpt2"
        elif (pre.get("type") == "Sequence" and len(pre.get("pretokenizers", [])) == 2
              and pre["pretokenizers"][0].get("type") == "Split"
              and pre["pretokenizers"][0].get("pattern", {}).get("Regex") == LLAMA3_SPLIT
              and pre["pretokenizers"][1].get("type") == "ByteLevel"
              and not pre["pretokenizers"][1].get("use_regex", True)
              and not pre["pretokenizers"][1].get("add_prefix_space")):
            mode = "llama3"
        else:
            return None
        merges = [tuple(x) if isinstance(x, list) else tuple(x.split(" ", 1)) for x in m["merges"]]
        added = [(a["content"], int(a["id"]), bool(a.get("special"))) for a in d.get("added_tokens", [])]
        enc = nrt.load().BpeTokenizer(m["vocab"], merges, added, mode, bool(m.get("ignore_merges")))
        for p in _PROBES:
            if enc.encode(p) != hf_tok.encode(p, add_special_tokens=False).ids:
                return None
        return enc
    except Exception:  # pragma: no cover - fall back to the HF encoder
        return None


class Tokenizer:
    """Thin wrapper with the few calls the engine needs.  Encoding runs on the native
    BPE encoder when it supports the tokenizer (token-for-token equal to HF; GIL
    released, multi-threaded batches), decoding on HF ``tokenizers``."""

    def __init__(self, hf_tok, kind: str = "builtin", native: bool = True):
        self.tok = hf_tok
        self.kind = kind
        self.native = native_encoder(hf_tok) if native and os.environ.get("LK_NATIVE_TOKENIZER", "1") != "0" else None
        self.vocab_size = hf_tok.get_vocab_size()
        v = hf_tok.get_vocab()
        self.bos_id = v.get("<|begin_of_text|>", v.get("<s>", v.get("[CLS]", 0)))
        self.eot_id = v.get("<|eot_id|>", v.get("</s>", v.get("[SEP]", 0)))
        self.eos_ids = {i for i in (v.get("<|end_of_text|>"), v.get("<|eot_id|>"), v.get("</s>")) if i is not None}
        self.cls_id = v.get("[CLS]", self.bos_id)
        self.sep_id = v.get("[SEP]", self.eot_id)
        self._piece_cache: Optional[list] = None

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        if self.native is not None:
            ids = self.native.encode(text)  # thread-safe: its word cache sits behind a shared mutex
        else:
            ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] + ids) if add_bos else ids

    def encode_batch(self, texts: Iterable[str]) -> list[list[int]]:
        texts = list(texts)
        if self.native is not None:
            return self.native.encode_batch(texts, min(8, max(1, len(texts) // 4)))
        return [e.ids for e in self.tok.encode_batch(texts, add_special_tokens=False)]

    def encode_for_embedding(self, texts: list[str], max_len: int = 512) -> list[list[int]]:
        """[CLS] text [SEP], truncated (BERT-style)."""
        out = []
        for ids in self.encode_batch(texts):
            ids = ids[: max_len - 2]
            out.append([self.cls_id] + ids + [self.sep_id])
        return out

    def decode(self, ids: list[int], skip_special: bool = True) -> str:
        ids = [i for i in ids if 0 <= i < self.vocab_size]
        return self.tok.decode(ids, skip_special_tokens=skip_special)

    def token_bytes_table(self) -> Optional[list]:
        """Raw bytes of every token id for byte-level BPE tokenizers (None otherwise): lets
        :class:`IncrementalDetokenizer` stream text in O(1) per token instead of re-decoding
        the whole output.  Special tokens map to b"" (decode skips them)."""
        if getattr(self, "_bytes_table", False) is not False:
            return self._bytes_table
        table = None
        try:
            import json as _json

            dec = _json.loads(self.tok.to_str()).get("decoder") or {}
            if dec.get("type") == "ByteLevel":
                b2u = _bytes_to_unicode()
                u2b = {u: b for b, u in b2u.items()}
                special = {t.content for t in self.tok.get_added_tokens_decoder().values() if t.special}
                table = []
                for i in range(self.vocab_size):
                    t = self.tok.id_to_token(i)
                    if t is None or t in special:
                        table.append(b"")
                    else:
                        table.append(bytes(u2b[c] for c in t) if all(c in u2b for c in t) else t.encode("utf-8"))
        except Exception:  # pragma: no cover - any tokenizer shape we do not understand
            table = None
        self._bytes_table = table
        return table

    def piece(self, i: int) -> str:
        """Decoded text of a single token (for constrained decoding)."""
        if self._piece_cache is None:
            self._piece_cache = [self.tok.decode([j], skip_special_tokens=False) for j in range(self.vocab_size)]
        return self._piece_cache[i] if 0 <= i < self.vocab_size else ""

    def special(self, name: str) -> int:
        return self.tok.token_to_id(name)

    # ------------------------------------------------------------ chat formats
    def chat_prompt(self, prompt: str, system: Optional[str] = None, style: str = "llama3") -> list[int]:
        """Token ids of the model's chat template around a raw /api/generate prompt."""
        if style == "raw":
            return self.encode(prompt, add_bos=True)
        sh, eh, eot = self.special("<|start_header_id|>"), self.special("<|end_header_id|>"), self.eot_id
        ids = [self.bos_id]
        if system:
            ids += [sh] + self.encode("system") + [eh] + self.encode("\n\n" + system) + [eot]
        ids += [sh] + self.encode("user") + [eh] + self.encode("\n\n" + prompt) + [eot]
        ids += [sh] + self.encode("assistant") + [eh] + self.encode("\n\n")
        return ids

    def chat_prompt_batch(self, prompts: list, system: Optional[str] = None, style: str = "llama3") -> list:
        """Batched :meth:`chat_prompt` (one parallel encode of all bodies)."""
        if style == "raw":
            return [[self.bos_id] + ids for ids in self.encode_batch(prompts)]
        sh, eh, eot = self.special("<|start_header_id|>"), self.special("<|end_header_id|>"), self.eot_id
        head = [self.bos_id]
        if system:
            head += [sh] + self.encode("system") + [eh] + self.encode("\n\n" + system) + [eot]
        head += [sh] + self.encode("user") + [eh]
        tail = [eot, sh] + self.encode("assistant") + [eh] + self.encode("\n\n")
        bodies = self.encode_batch(["\n\n" + p for p in prompts])
        return [head + b + tail for b in bodies]


def _bytes_to_unicode() -> dict:
    """GPT-2 / Llama-3 byte-level BPE alphabet: byte -> printable unicode character."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class IncrementalDetokenizer:
    """Streams text for growing id lists without re-decoding emitted text and without
    splitting multi-byte UTF-8 characters across chunks.  Byte-level tokenizers take the
    O(1)-per-token path (token bytes -> incremental UTF-8 decoder); others re-decode."""

    def __init__(self, tok: Tokenizer):
        import codecs

        self.tok = tok
        self.ids: list[int] = []
        self.sent = ""
        tb = tok.token_bytes_table() if hasattr(tok, "token_bytes_table") else None
        self.table = tb
        self.udec = codecs.getincrementaldecoder("utf-8")("replace") if tb is not None else None

    def push(self, tid: int) -> str:
        if self.table is not None:
            return self.udec.decode(self.table[tid]) if 0 <= tid < len(self.table) else ""
        self.ids.append(tid)
        text = self.tok.decode(self.ids)
        if text.endswith("�"):
            return ""
        new = text[len(self.sent):]
        self.sent = text
        return new


_builtin: Optional[Tokenizer] = None


def builtin_tokenizer() -> Tokenizer:
    global _builtin
    with _lock:
        if _builtin is None:
            from tokenizers import Tokenizer as HFTok

            if _CACHE.exists():
                hf = HFTok.from_file(str(_CACHE))
            else:
                hf = _train_builtin()
                try:
                    _CACHE.parent.mkdir(parents=True, exist_ok=True)
                    tmp = _CACHE.with_suffix(f".{os.getpid()}.tmp")
                    hf.save(str(tmp))
                    os.replace(tmp, _CACHE)
                except OSError:
                    pass
            _builtin = Tokenizer(hf, "builtin")
    return _builtin


def load_tokenizer(path: Optional[str] = None) -> Tokenizer:
    if path:
        p = Path(path)
        f = p / "tokenizer.json" if p.is_dir() else p
        if f.exists():
            from tokenizers import Tokenizer as HFTok

            return Tokenizer(HFTok.from_file(str(f)), "hf")
    return builtin_tokenizer()


def describe(tok: Tokenizer) -> dict:
    return {"kind": tok.kind, "vocab_size": tok.vocab_size, "bos": tok.bos_id, "eot": tok.eot_id}


if __name__ == "__main__":  # pragma: no cover
    t = builtin_tokenizer()
    print(json.dumps(describe(t)))

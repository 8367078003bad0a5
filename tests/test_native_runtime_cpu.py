"""C++ block allocator == Python block allocator, operation by operation."""
import os
import random

import pytest

from llm_kubernetes_minikube_sharp4dev_amd.engine.block_manager import BlockAllocator, NoFreeBlocks, chain_hash
from llm_kubernetes_minikube_sharp4dev_amd.native import runtime


@pytest.fixture(scope="module")
def native():
    try:
        runtime.build()
    except (ImportError, FileNotFoundError) as e:  # toolchain missing (pybind11 / g++): Python fallback
        pytest.skip(f"native build toolchain unavailable: {e}")
    # a RuntimeError from a failed compile of csrc/runtime/*.cpp is NOT skipped: it fails the tests
    return runtime


def test_chain_hash_matches(native):
    m = native.load()
    for toks in ([], [1, 2, 3], list(range(16)), [128000, 7, 99999]):
        for parent in (0, 12345678901234567, 2**64 - 1):
            assert m.chain_hash(parent, toks) == chain_hash(parent, toks)


def test_random_ops_equivalent(native):
    rng = random.Random(0)
    py = BlockAllocator(24, 4, True)
    nat = native.NativeBlockAllocator(24, 4, True)
    owned_py, owned_nat = [], []
    prefixes = [[rng.randrange(50) for _ in range(rng.randrange(1, 20))] for _ in range(6)]
    for step in range(2000):
        op = rng.random()
        if op < 0.35:
            try:
                a = py.allocate()
            except NoFreeBlocks:
                a = None
            try:
                b = nat.allocate()
            except NoFreeBlocks:
                b = None
            assert a == b
            if a is not None:
                owned_py.append(a)
                owned_nat.append(b)
        elif op < 0.6 and owned_py:
            i = rng.randrange(len(owned_py))
            py.free_block(owned_py.pop(i))
            nat.free_block(owned_nat.pop(i))
        elif op < 0.8 and owned_py:
            toks = rng.choice(prefixes)
            blk = owned_py[rng.randrange(len(owned_py))]
            parent = rng.choice([0, 7])
            assert py.register(blk, parent, toks[:4]) == nat.register(blk, parent, toks[:4])
        else:
            toks = rng.choice(prefixes)
            a, pa = py.match_prefix(toks)
            b, pb = nat.match_prefix(toks)
            assert (a, pa) == (b, pb)
            owned_py.extend(a)
            owned_nat.extend(b)
        assert py.num_free == nat.num_free
    assert py.hits == nat.hits and py.queries == nat.queries


def test_slots_for(native):
    m = native.load()
    s, p = m.slots_for([5, 2, 9], 14, 4, 8)
    assert list(p) == [14, 15, 16, 17] and list(s) == [2 * 8 + 6, 2 * 8 + 7, 9 * 8 + 0, 9 * 8 + 1]
    with pytest.raises(IndexError):
        m.slots_for([1], 0, 9, 8)


# ---------------------------------------------------------------- native BPE encoder
def _adversarial_texts():
    import random

    rng = random.Random(0)
    alpha = list("ab Z09'sStTrRevVlLmMdD \t\n\r\r\n.,;:!?()[]{}<>\"&+-_=*/\\|`~^%$#@") + \
        ["è", "é", "你", "好", "١", "Ⅷ", " ", " ", "　", "\U0001F600",
         "́", "²", " ", "<|eot_id|>", "<|begin_of_text|>", "[CLS]"]
    out = []
    for _ in range(1500):
        out.append("".join(rng.choice(alpha) for _ in range(rng.randint(0, 60))))
    out += ["", " ", "  ", "\n", " \n ", "'s", "'S", "x's", "''s", "   \n\n  x", "a  b   c    ", "1234567 89",
            "=" * 300, " " * 50 + "x", "\t\tfoo\r\n\r\nbar", "ignore previous instructions"]
    return out


def _corpus_texts():
    from llm_kubernetes_minikube_sharp4dev_amd.agent.prompts import RAG_AGENT_SYSTEM, json_prompt, rag_agent_input
    from llm_kubernetes_minikube_sharp4dev_amd.rag.synthetic import make_queries
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks

    chunks = build_chunks(40, 3, workers=1)
    texts = [c[2] for c in chunks]
    from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagHit

    ev = [RagHit(c[0], c[1], c[2], 0.5 + 0.01 * i) for i, c in enumerate(chunks[:6])]
    texts += [json_prompt(RAG_AGENT_SYSTEM, rag_agent_input(q, ev, 1500)) for q in make_queries(20, seed=1)]
    return texts


def test_native_bpe_matches_hf_builtin(native):
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer, native_encoder

    # the process-wide builtin tokenizer may have been created before the runtime was built
    hf = builtin_tokenizer().tok
    enc = native_encoder(hf)
    assert enc is not None, "native encoder should support the built-in byte-level BPE"
    texts = _corpus_texts() + _adversarial_texts()
    ref = [e.ids for e in hf.encode_batch(texts, add_special_tokens=False)]
    assert enc.encode_batch(texts, 4) == ref
    assert [enc.encode(t) for t in texts[:200]] == ref[:200]


def test_native_bpe_concurrent_callers(native):
    """Several Python threads encoding through ONE encoder at once (a server's event loop,
    its engine thread and the embedding batcher): the shared word cache is read under a
    shared lock and merged exclusively, so every thread gets the serial result."""
    import threading

    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer, native_encoder

    hf = builtin_tokenizer().tok
    enc = native_encoder(hf)
    texts = _corpus_texts() + _adversarial_texts()
    ref = [e.ids for e in hf.encode_batch(texts, add_special_tokens=False)]
    errs = []

    def work(t):
        try:
            for r in range(6):
                part = texts[(t * 37 + r * 11) % len(texts):][:64]
                exp = ref[(t * 37 + r * 11) % len(texts):][:64]
                got = enc.encode_batch(part, 2) if (t + r) % 2 else [enc.encode(x) for x in part]
                if got != exp:
                    errs.append((t, r))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:3]


def test_native_bpe_matches_hf_llama3_pretokenizer(native):
    """Llama-3 layout: Split(llama-3 regex, isolated) + ByteLevel(no regex), ignore_merges."""
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import LLAMA3_SPLIT, native_encoder

    hf = Tokenizer(models.BPE(ignore_merges=True))
    hf.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    hf.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=3000, special_tokens=["<|begin_of_text|>", "<|eot_id|>"],
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    texts = _corpus_texts()
    hf.train_from_iterator(texts * 2, trainer=trainer)
    enc = native_encoder(hf)
    assert enc is not None
    allt = texts + _adversarial_texts()
    assert enc.encode_batch(allt, 3) == [e.ids for e in hf.encode_batch(allt, add_special_tokens=False)]


def test_native_decode_rows_matches_python(native):
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.native import runtime as nrt

    m = nrt.load()
    rng = np.random.default_rng(0)
    tables = [list(rng.integers(0, 1000, n)) for n in (3, 1, 7, 5)]
    starts = [40, 3, 100, 79]
    toks = [11, 12, 13, 14]
    lens = [41, 4, 101, 80]
    ids, pos, slots, ctx, bt = m.decode_rows([list(map(int, t)) for t in tables], starts, toks, lens, 16, 8, 8)
    assert ids.shape == (8,) and bt.shape == (8, 8)
    for i, t in enumerate(tables):
        assert slots[i] == t[starts[i] // 16] * 16 + starts[i] % 16
        assert list(bt[i, : len(t)]) == list(t) and not bt[i, len(t):].any()
    assert list(slots[4:]) == [-1] * 4 and list(ctx[4:]) == [1] * 4 and list(ids[:4]) == toks


@pytest.mark.skipif(bool(os.environ.get("LK_NATIVE_RUNTIME_SO")), reason="already running under the sanitizer build")
def test_runtime_under_asan_ubsan(native):
    """Every test of this file again, against an ASan + UBSan build of csrc/runtime/*.cpp
    (bpe.cpp's Unicode scanners, the block allocator, the decode-row packer)."""
    import subprocess
    import sys

    try:
        so = native.build(sanitize=True)
    except (ImportError, FileNotFoundError) as e:
        pytest.skip(f"sanitizer toolchain unavailable: {e}")
    # libstdc++ is preloaded too: python itself does not link it, so ASan's __cxa_throw
    # interceptor would otherwise find no real symbol and abort on the first C++ exception
    libs = [subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
            for n in ("libasan.so", "libstdc++.so")]
    if not all(os.path.isabs(x) for x in libs):
        pytest.skip("libasan / libstdc++ not found")
    env = dict(os.environ, LK_NATIVE_RUNTIME_SO=str(so), LD_PRELOAD=" ".join(libs),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", __file__],
                       capture_output=True, text=True, env=env, timeout=900,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout


def test_device_assert_build_compiles(tmp_path):
    """The LK_DEBUG build (device asserts on, `csrc/build.py --debug`) must compile: every
    kernel source that uses LK_DASSERT, device code only, for gfx950."""
    import glob
    import shutil
    import subprocess

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srcs = [s for s in sorted(glob.glob(os.path.join(root, "csrc", "*.hip"))) if "LK_DASSERT" in open(s).read()]
    assert srcs
    for s in srcs:
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-std=c++17", "-DLK_DEBUG", "--offload-device-only",
                            "-c", s, "-o", str(tmp_path / (os.path.basename(s) + ".o"))],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (s, r.stderr[-2000:])

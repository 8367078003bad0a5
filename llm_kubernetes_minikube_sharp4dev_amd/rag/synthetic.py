"""Deterministic synthetic runbook corpora (BASELINE.json: "synthetic corpora").

Documents look like the reference's knowledge base (``knowledge/runbook_scaling.md``):
optional YAML front-matter with ``allowed_namespaces`` / ``tool_hints``, Markdown
sections, numbered procedures mentioning the agent tools — mixed Italian/English
DevOps prose, so chunk lengths, header splits and tokenizer ratios are realistic.
"""
from __future__ import annotations

import random
from typing import Iterator

TOPICS = [
    ("scaling", "Scaling sicuro di un Deployment", ["scaling", "deployment", "hpa"]),
    ("logs", "Analisi dei log di un Pod", ["logs", "troubleshooting"]),
    ("rollout", "Rollout e rollback di una release", ["rollout", "deployment"]),
    ("network", "Diagnosi di problemi di rete nel cluster", ["network", "service", "dns"]),
    ("storage", "Gestione dei PersistentVolume", ["storage", "pvc"]),
    ("nodes", "Manutenzione dei nodi", ["nodes", "drain", "cordon"]),
    ("secrets", "Rotazione dei Secret", ["security", "secrets"]),
    ("quota", "ResourceQuota e LimitRange", ["quota", "limits"]),
    ("ingress", "Configurazione Ingress e certificati", ["ingress", "tls"]),
    ("jobs", "CronJob e Job batch", ["jobs", "batch"]),
]
NAMESPACES = ["dev", "staging", "sharp4dev", "test-ns-giovanni", "prod", "default", "monitoring"]
TOOLS = ["cluster_context", "list_pods", "get_logs", "scale_deployment", "final_answer"]
WORDS = (
    "il pod deployment namespace replica cluster nodo servizio readiness liveness probe container "
    "immagine rollout rollback metrica soglia allarme latenza memoria cpu richiesta limite quota "
    "verificare applicare controllare attendere ripristinare aumentare ridurre monitorare annotare "
    "the pod should be ready before traffic is routed check the events and the restart count "
    "kubectl describe get logs scale rollout status undo apply delete cordon drain uncordon "
    "entro minuti secondi percentuale stato sintetico incremento massimo approvazione ticket "
    "operatore turno reperibilita incidente postmortem causa radice mitigazione escalation "
    "configmap secret volume claim storageclass ingress service endpoint selector label annotation "
    "horizontal pod autoscaler target utilization resource requests limits eviction pressure oom "
    "when the error rate exceeds the threshold roll back to the previous revision immediately"
).split()


_SYL = ("ca co cu ra re ri ro ta te ti to pa pe pi po la le li lo ma me mi mo na ne ni no sa se "
        "si so va ve vi za zo gli gna chi che sta sto stre tra tro pro pre con per ver zio ne").split()


def _lexicon(n: int = 6000, seed: int = 99) -> list[str]:
    """Open, Zipf-sampled vocabulary of Italian-like pseudo-words (so BPE statistics
    and chars/token ratios resemble natural text instead of a closed word list)."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        w = "".join(rng.choice(_SYL) for _ in range(rng.choice((1, 2, 2, 3, 3, 4))))
        out.append(w + rng.choice(("", "", "o", "a", "e", "i", "mente", "zione")))
    return out


LEXICON = _lexicon()


def _word(rng: random.Random) -> str:
    if rng.random() < 0.45:
        return rng.choice(WORDS)
    # Zipf-ish rank sampling
    r = int(len(LEXICON) * (rng.random() ** 2.5))
    return LEXICON[min(r, len(LEXICON) - 1)]


def _sentence(rng: random.Random, n_min=8, n_max=22) -> str:
    n = rng.randint(n_min, n_max)
    s = " ".join(_word(rng) for _ in range(n))
    return s[0].upper() + s[1:] + "."


def _long_section(rng: random.Random, title: str, chars: int) -> str:
    body = []
    while len(title) + sum(len(b) + 1 for b in body) < chars:
        body.append(_sentence(rng))
    text = f"## {title}\n" + " ".join(body)
    return text[:chars].rstrip() + ".\n"


def make_document(i: int, seed: int = 0, target_chars: int = 1200, section_chars: int = 0) -> str:
    """One runbook.  ``section_chars`` > 0: the long-evidence regime -- every section grown to
    about that many characters (set it just under the 1200-char header-split cap of
    ``RagIndex.cs:92-95`` so each section stays ONE chunk, and the /agent_rag prompt carries
    6 evidence chunks near the 1500-char evidence cap of ``Minimal_RAG/Program.cs:159``)."""
    rng = random.Random(seed * 1_000_003 + i)
    if section_chars > 0:
        slug, title, tags = TOPICS[i % len(TOPICS)]
        secs = [f"---\ntitle: \"{title} #{i}\"\nslug: \"{slug}-{i}\"\nallowed_namespaces: [\"dev\", \"staging\"]\n---\n"]
        for name in ("Obiettivo", "Procedura", "Note operative", "Verifiche", "Rollback"):
            secs.append(_long_section(rng, f"{name} ({slug})", section_chars))
        return "\n".join(secs)
    slug, title, tags = TOPICS[i % len(TOPICS)]
    parts = []
    if rng.random() < 0.5:
        ns = rng.sample(NAMESPACES[:4], rng.randint(1, 4))
        hints = rng.sample(TOOLS[:4], 2)
        parts.append(
            "---\n"
            f'title: "{title} #{i}"\n'
            f'slug: "{slug}-{i}"\n'
            f"tags: {tags}\n".replace("'", '"')
            + f'severity: "{rng.choice(["low", "medium", "high"])}"\n'
            + "allowed_namespaces: [" + ", ".join(f'"{n}"' for n in ns) + "]\n"
            + "tool_hints:\n"
            + "".join(f'  - tool: "{h}"\n    when: "{_sentence(rng, 4, 8)}"\n' for h in hints)
            + f'updated_at: "2025-0{rng.randint(1, 9)}-1{rng.randint(0, 9)}"\n---\n'
        )
    parts.append(f"## Obiettivo\n{_sentence(rng)} {_sentence(rng)}\n")
    steps = []
    for k in range(rng.randint(2, 5)):
        tool = rng.choice(TOOLS[:4])
        steps.append(f"{k + 1}. **Passo {k + 1}**: `{tool}` {_sentence(rng, 6, 14)}")
    parts.append("## Procedura sintetica\n" + "\n".join(steps) + "\n")
    body = []
    while sum(len(p) for p in parts) + sum(len(b) for b in body) < target_chars:
        body.append(_sentence(rng))
    parts.append("## Note operative\n" + " ".join(body) + "\n")
    parts.append(f"## Rollback\n- {_sentence(rng, 6, 12)}\n")
    return "\n".join(parts)


def iter_documents(n: int, seed: int = 0, min_chars: int = 400, max_chars: int = 2400) -> Iterator[tuple[str, str]]:
    rng = random.Random(seed)
    for i in range(n):
        slug = TOPICS[i % len(TOPICS)][0]
        yield f"runbook_{slug}_{i:07d}.md", make_document(i, seed, rng.randint(min_chars, max_chars))


def make_queries(n: int, seed: int = 0, unique: bool = True) -> list[str]:
    """Agent requests in the style of the demo videos (scale / list / logs / status).
    ``unique`` appends a distinct ticket reference so no two requests of a benchmark
    share a whole prompt (only the system-prompt prefix is shared)."""
    rng = random.Random(seed + 17)
    templates = [
        "Scala il deployment {d} nel namespace {ns} a {r} repliche",
        "Mostrami i pod nel namespace {ns}",
        "Recupera i log del pod {d}-{h} nel namespace {ns}",
        "Qual e lo stato del cluster?",
        "Porta {d} a {r} repliche in {ns} seguendo il runbook di scaling",
        "Perche il pod {d}-{h} in {ns} continua a riavviarsi?",
    ]
    out = []
    for _ in range(n):
        t = rng.choice(templates)
        q = t.format(d=rng.choice(["echoserver", "api", "web", "worker"]),
                     ns=rng.choice(NAMESPACES), r=rng.randint(1, 10),
                     h=f"{rng.randint(0, 0xfffff):05x}")
        if unique:
            q += f" (ticket INC-{seed & 0xffffff:06x}-{len(out):04d}, {_sentence(rng, 3, 9).lower()})"
        out.append(q)
    return out


def training_text(n_docs: int = 40, seed: int = 0) -> list[str]:
    """Text used to train the built-in byte-level BPE tokenizer: synthetic runbooks,
    agent queries, and (when present) English prose from the Python stdlib
    docstrings of the image, for realistic subword statistics."""
    import glob
    import re
    import sys

    docs = [d for _, d in iter_documents(n_docs, seed)]
    prose = []
    libdir = f"{sys.base_prefix}/lib/python{sys.version_info.major}.{sys.version_info.minor}"
    for f in sorted(glob.glob(libdir + "/*.py"))[:400]:
        try:
            src = open(f, encoding="utf-8", errors="ignore").read()
        except OSError:
            continue
        prose.extend(m.group(1) for m in re.finditer(r'"""(.*?)"""', src, re.S))
    return docs + make_queries(2000, seed) + prose

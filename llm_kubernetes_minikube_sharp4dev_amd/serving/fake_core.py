"""A protocol-exact stand-in for an engine core (:mod:`.engine_core`) with no model: every
``gen`` request receives ``tokens`` token ids, one per simulated engine step of ``step_s``
seconds, batched per step and connection exactly like the real core's frames.  For load
tests of the HTTP front-ends / routing (``benchmarks/frontend_load.py``) and CPU tests: it
isolates the serving path's own cost from GPU work."""
from __future__ import annotations

import asyncio
import os
import struct

import msgpack
import numpy as np

_HDR = struct.Struct("<I")


class FakeCore:
    def __init__(self, path: str, tokens: int = 48, step_s: float = 0.002, dim: int = 768, vocab: int = 32000):
        self.path, self.tokens, self.step_s, self.dim, self.vocab = path, tokens, step_s, dim, vocab
        self.served = 0
        self.aborted = 0
        self._server = None

    async def start(self):
        if os.path.exists(self.path):
            os.unlink(self.path)
        self._server = await asyncio.start_unix_server(self._conn, path=self.path, limit=1 << 24)

    async def _conn(self, reader, writer):
        active: dict = {}  # rid -> tokens left
        lock = asyncio.Lock()

        def send(obj):
            body = msgpack.packb(obj, use_bin_type=True)
            writer.write(_HDR.pack(len(body)) + body)

        async def stepper():
            while True:
                await asyncio.sleep(self.step_s)
                if not active:
                    continue
                items = []
                for rid in list(active):
                    left = active[rid] - 1
                    tid = 1000 + (rid * 7 + left) % 20000
                    if left <= 0:
                        del active[rid]
                        items.append([rid, [tid], True, "length", 0, None])
                        self.served += 1
                    else:
                        active[rid] = left
                        items.append([rid, [tid], False, None, None, None])
                send(["tok", items, [100000, 0, len(active)]])
                await writer.drain()

        task = asyncio.get_running_loop().create_task(stepper())
        try:
            while True:
                n = _HDR.unpack(await reader.readexactly(4))[0]
                msg = msgpack.unpackb(await reader.readexactly(n), raw=False)
                op, rid = msg[0], msg[1]
                if op == "gen":
                    sp = msg[4]
                    active[rid] = min(self.tokens, int(sp.get("max_tokens") or self.tokens))
                elif op == "abort":
                    if active.pop(rid, None) is not None:
                        self.aborted += 1
                elif op == "load":
                    send(["load", rid, {"kind": "generate" if "embed" not in msg[2] else "embed", "name": msg[2],
                                        "preset": msg[2], "max_model_len": 8192, "eos_ids": [], "chat_style": "llama3",
                                        "load_s": 0.0, "vocab_size": self.vocab}])
                elif op == "embed":
                    v = np.ones((len(msg[3]), self.dim), np.float32) / np.sqrt(self.dim)
                    send(["emb", rid, v.tobytes(), v.shape[0], v.shape[1]])
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            task.cancel()
            writer.close()


async def serve(paths: list[str], tokens: int = 48, step_s: float = 0.002):
    cores = [FakeCore(p, tokens, step_s) for p in paths]
    for c in cores:
        await c.start()
    return cores


def main():  # python -m llm_kubernetes_minikube_sharp4dev_amd.serving.fake_core PATH[,PATH...] [tokens] [step_s]
    import sys

    paths = sys.argv[1].split(",")
    tokens = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    step_s = float(sys.argv[3]) if len(sys.argv) > 3 else 0.002

    async def run():
        await serve(paths, tokens, step_s)
        await asyncio.Event().wait()

    asyncio.run(run())


if __name__ == "__main__":
    main()

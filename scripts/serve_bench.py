"""Serving throughput of the consensus server's engines (``server.ConsensusService``) on one GPU:
R consensus requests issued by C concurrent clients against warm engines. With C > 1 requests for
the same responder engine decode as one batch (weights read once per step for every row) and the
judge sessions that finish together decode as one batch, so aggregate tokens/s grows with C while
per-request latency grows much less.

  python scripts/serve_bench.py --models llama-3-8b@0,llama-3-8b@1 --judge llama-3-8b@judge \\
      --concurrency 1,4 --requests 4 --max-tokens 512
"""
import argparse
import os
import random
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_consensus_amd.context import Context  # noqa: E402
from llm_consensus_amd.server import ConsensusService  # noqa: E402
from llm_consensus_amd.utils.tokenizer import get_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama-3-8b@0,llama-3-8b@1")
    ap.add_argument("--judge", default="llama-3-8b@judge")
    ap.add_argument("--concurrency", default="1,4")
    ap.add_argument("--requests", type=int, default=4)
    ap.add_argument("--max-tokens", type=int, default=512)
    ap.add_argument("--prompt-tokens", type=int, default=128)
    a = ap.parse_args()

    models = [m for m in a.models.split(",") if m]
    tok = get_tokenizer(128256)
    rng = random.Random(1234)
    prompts = [tok.decode([rng.randrange(256, 60000) for _ in range(a.prompt_tokens)]).strip() for _ in range(64)]

    for conc in [int(c) for c in a.concurrency.split(",")]:
        t0 = time.monotonic()
        svc = ConsensusService(models, a.judge, concurrency=conc, max_tokens=a.max_tokens, timeout=3600)
        print(f"C={conc}: engines ready in {time.monotonic() - t0:.1f}s", flush=True)
        try:
            # warm-up request (first-touch allocations)
            svc.run(Context.background(), svc.parse({"prompt": prompts[0], "max_tokens": 16}))
            lat, toks = [], [0]
            lock = threading.Lock()
            nxt = [0]

            def client():
                while True:
                    with lock:
                        i = nxt[0]
                        nxt[0] += 1
                    if i >= a.requests:
                        return
                    s = time.monotonic()
                    res = svc.run(Context.background(), svc.parse({"prompt": prompts[i % len(prompts)]}))
                    el = time.monotonic() - s
                    n = sum(r.output_tokens for r in res.responses)
                    # judge tokens: re-tokenized consensus length (passthrough adds none)
                    n += len(tok.encode(res.consensus)) if len(res.responses) > 1 else 0
                    with lock:
                        lat.append(el)
                        toks[0] += n

            t = time.monotonic()
            ths = [threading.Thread(target=client) for _ in range(conc)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            wall = time.monotonic() - t
            print(f"C={conc}: {a.requests} requests x ({len(models)} responders + judge) x {a.max_tokens} tokens in "
                  f"{wall:.2f}s -> {toks[0] / wall:.1f} output tokens/s aggregate, p50 request latency "
                  f"{statistics.median(lat):.2f}s", flush=True)
        finally:
            svc.close()


if __name__ == "__main__":  # worker processes are spawned: no work at import
    main()

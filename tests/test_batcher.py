"""Continuous batching (engine/batcher.py): rows join and leave between replays; every request
must get exactly the tokens it gets when decoded alone (greedy and seeded sampling), whatever
rows it shared the batch with and wherever compaction moved it."""

import pytest
import torch

from llm_consensus_amd.engine import Engine, EngineConfig, SamplingParams
from llm_consensus_amd.engine.batcher import ContinuousBatcher
from llm_consensus_amd.models.config import FAMILIES


def _engine(device, max_batch=3):
    return Engine(FAMILIES["llama-tiny"], EngineConfig(device=device, max_context=512, max_batch=max_batch,
                                                       max_seqs=6, seed=11))


def _alone(eng, prompt, p):
    s = eng.new_sequence()
    eng.prefill([s], [prompt])
    out = eng.decode([s], [p])[0]
    eng.free_sequence(s)
    return out


def _run_schedule(eng, reqs, admit_at):
    """reqs: [(prompt, params)]; admit_at[i] = step index at which request i is admitted."""
    bat = ContinuousBatcher(eng)
    done = {}
    step, pending = 0, list(range(len(reqs)))
    while pending or bat.rows:
        for i in [i for i in pending if admit_at[i] <= step and bat.free_rows]:
            s = eng.new_sequence()
            eng.prefill([s], [reqs[i][0]])
            bat.admit(s, reqs[i][1], tag=i)
            pending.remove(i)
        for row in bat.step():
            assert row.error is None
            done[row.tag] = row.tokens
            eng.free_sequence(row.seq)
        step += 1
    return [done[i] for i in range(len(reqs))]


def _check(device):
    eng = _engine(device)
    reqs = [
        ([300 + i for i in range(40)], SamplingParams(max_tokens=40, temperature=0.0, stop_on_eos=False)),
        ([500 + i for i in range(9)], SamplingParams(max_tokens=7, temperature=0.0, stop_on_eos=False)),
        ([700 + 3 * i for i in range(23)], SamplingParams(max_tokens=30, temperature=1.0, seed=5, stop_on_eos=False)),
        ([100 + i for i in range(5)], SamplingParams(max_tokens=12, temperature=0.8, top_k=20, seed=9,
                                                     stop_on_eos=False)),
    ]
    free0 = eng.alloc.num_free
    ref = [_alone(eng, p, sp) for p, sp in reqs]
    # 0 and 1 start together; 1 retires first; 2 joins mid-flight; 0 retires -> 2 moves down; 3
    # joins after the batch was full
    got = _run_schedule(eng, reqs, admit_at=[0, 0, 2, 3])
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, (i, g, r)
        assert len(g) == reqs[i][1].max_tokens
    assert eng.alloc.num_free == free0  # every retired row's KV blocks came back


def test_continuous_batching_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_continuous_batching_gpu(cuda):
    _check("cuda:0")


def test_continuous_batching_cancelled_row_cpu():
    """A row whose request is cancelled mid-decode is retired with the context's error; the rows
    around it (moved by compaction) still get their solo tokens."""
    from llm_consensus_amd.context import Context, ContextError

    eng = _engine("cpu")
    reqs = [([300 + i for i in range(12)], SamplingParams(max_tokens=30, temperature=0.0, stop_on_eos=False)),
            ([400 + i for i in range(7)], SamplingParams(max_tokens=30, temperature=0.0, stop_on_eos=False)),
            ([500 + i for i in range(9)], SamplingParams(max_tokens=25, temperature=0.0, stop_on_eos=False))]
    ref = [_alone(eng, p, sp) for p, sp in reqs]
    bat = ContinuousBatcher(eng)
    ctxs = [Context.background() for _ in reqs]
    for i, (p, sp) in enumerate(reqs):
        s = eng.new_sequence()
        eng.prefill([s], [p])
        bat.admit(s, sp, tag=i, ctx=ctxs[i])
    done, step = {}, 0
    while bat.rows:
        if step == 1:
            ctxs[0].cancel()  # row 0: the others move down when it retires
        for row in bat.step():
            done[row.tag] = row
            eng.free_sequence(row.seq)
        step += 1
    assert isinstance(done[0].error, ContextError)
    for i in (1, 2):
        assert done[i].error is None and done[i].tokens == ref[i]


@pytest.mark.gpu
def test_batching_engine_long_rows_batch_invariant(cuda):
    """A batching engine (16 rows x 2 kv heads: the length-only attention split, min 2048 keys per
    block) over rows of very different lengths: a 3000-key row (two split ranges) decoded beside
    short rows, whose batch selects larger buckets than they would alone, still gets exactly its
    solo tokens, and so do they."""
    eng = Engine(FAMILIES["llama-tiny"], EngineConfig(device="cuda:0", max_context=4000, max_batch=16, max_seqs=6,
                                                      seed=13))
    reqs = [
        ([(7 * i) % 900 + 100 for i in range(3000)], SamplingParams(max_tokens=24, temperature=0.0, stop_on_eos=False)),
        ([500 + i for i in range(9)], SamplingParams(max_tokens=20, temperature=0.0, stop_on_eos=False)),
        ([(11 * i) % 800 + 150 for i in range(2100)], SamplingParams(max_tokens=16, temperature=1.0, seed=3,
                                                                     stop_on_eos=False)),
        ([100 + i for i in range(5)], SamplingParams(max_tokens=12, temperature=0.0, stop_on_eos=False)),
    ]
    ref = [_alone(eng, p, sp) for p, sp in reqs]
    got = _run_schedule(eng, reqs, admit_at=[0, 0, 1, 2])
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, (i, g, r)


@pytest.mark.gpu
def test_three_rows_eight_kv_heads_batch_invariant(cuda):
    """3 rows x 8 kv heads (3 duplicate 8B responders batched in one engine: 24 (row, head)
    units, the length-only split with a 512-key minimum): rows of 2900, 9 and 1300 keys, whose
    batch selects larger attention buckets than the short rows would alone, get exactly their
    solo tokens (the bucket-dependent fused chunk used to change their rounding)."""
    cfg = FAMILIES["llama-tiny"].with_(name="llama-tiny-kv8", hidden=1024, n_heads=16, n_kv_heads=8, head_dim=64,
                                       intermediate=1024)
    eng = Engine(cfg, EngineConfig(device="cuda:0", max_context=4000, max_batch=3, max_seqs=6, seed=21))
    reqs = [
        ([(7 * i) % 900 + 100 for i in range(2900)], SamplingParams(max_tokens=24, temperature=0.0, stop_on_eos=False)),
        ([500 + i for i in range(9)], SamplingParams(max_tokens=20, temperature=1.0, seed=5, stop_on_eos=False)),
        ([(11 * i) % 800 + 150 for i in range(1300)], SamplingParams(max_tokens=16, temperature=0.0,
                                                                     stop_on_eos=False)),
    ]
    ref = [_alone(eng, p, sp) for p, sp in reqs]
    got = _run_schedule(eng, reqs, admit_at=[0, 0, 1])
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g == r, (i, g, r)


@pytest.mark.gpu
def test_attention_fault_fails_batched_rows(cuda):
    """A decode-attention merge that gave up (the kernel's fault word) fails the rows whose
    replays it covered, with an error, instead of streaming their tokens on."""
    eng = _engine("cuda:0")
    bat = ContinuousBatcher(eng)
    s = eng.new_sequence()
    eng.prefill([s], [[100 + i for i in range(20)]])
    row = bat.admit(s, SamplingParams(max_tokens=64, temperature=0.0, stop_on_eos=False))
    bat.step()
    eng.attn_fault.fill_(1)  # what a merger that gave up writes
    torch.cuda.synchronize()
    gone = []
    for _ in range(4):
        gone += bat.step()
        if gone:
            break
    assert gone == [row] and row.error is not None and "merge timed out" in str(row.error)
    torch.cuda.synchronize()  # the re-arm is queued on the engine's stream
    assert int(eng.attn_fault.item()) == 0


@pytest.mark.gpu
def test_attention_fault_in_flight_replay_is_not_lost(cuda):
    """A fault raised by the replay that is still in flight when the previous snapshot's fault is
    handled must not be wiped: a row admitted after that snapshot (so not in it) but decoded by
    the faulting replay fails too (the re-arm used to be queued behind that replay)."""
    eng = _engine("cuda:0")
    bat = ContinuousBatcher(eng)
    inject = {"on": True}
    real_graph = eng._graph

    class Faulting:
        def __init__(self, g):
            self.g = g

        def replay(self):
            self.g.replay()
            if inject["on"]:
                eng.attn_fault.fill_(1)  # on the engine stream, after the replay's kernels

    eng._graph = lambda B, bk: Faulting(real_graph(B, bk))
    sa, sb = eng.new_sequence(), eng.new_sequence()
    eng.prefill([sa], [[100 + i for i in range(20)]])
    eng.prefill([sb], [[200 + i for i in range(20)]])
    a = bat.admit(sa, SamplingParams(max_tokens=128, temperature=0.0, stop_on_eos=False))
    bat.step()                      # replay 1 faults; snapshot 1 carries it
    b = bat.admit(sb, SamplingParams(max_tokens=128, temperature=0.0, stop_on_eos=False))
    gone = bat.step()               # replay 2 (rows a, b) faults too; snapshot 1 fails a
    assert a in gone and a.error is not None
    inject["on"] = False
    for _ in range(3):
        gone += bat.step()
        if b in gone:
            break
    assert b in gone and b.error is not None and "merge timed out" in str(b.error)
    torch.cuda.synchronize()
    assert int(eng.attn_fault.item()) == 0

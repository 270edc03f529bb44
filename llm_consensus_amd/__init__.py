"""llm_consensus_amd — an MI355X-native multi-model consensus engine.

Same observable contract as johnayoung/llm-consensus (CLI flags, result.json schema,
``data/<run-id>/`` layout — reference ``cmd/llm-consensus/main.go``), but every "provider"
is a local model served by a PyTorch-ROCm engine whose hot ops are hand-written CDNA4 HIP
kernels (``csrc/kernels``), scheduled one process per GPU with RCCL over xGMI for TP.

Layer map:
  T7 cli.py / flags.py              CLI (Go ``flag`` semantics)
  T6 ui.py / output.py              presentation + Go-compatible JSON
  T5 runner.py / consensus.py       fan-out + judge
  T4 provider/                      Provider API, registry, stub + local providers
  T3 runtime/ parallel/placement.py worker-per-GPU control plane + placement solver
  T2 engine/                        prefill/decode engine, paged KV, sampler, HIP graphs
  T1 models/ parallel/              Llama-3 / Mixtral / Phi-3 + TP layers + comm
  T0 ops/ (+ csrc/)                 HIP kernels (gfx950, MFMA/LDS)
"""

from .version import __version__  # noqa: F401

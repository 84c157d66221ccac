"""Shared checks of the drop-in tests (the reference libllama on libggml-mi355x.so).

graph_splits(): libllama's scheduler summary, "graph splits = N" (src/llama-context.cpp:
523-533), which oracle/ref_llama_bench.cpp forwards to stderr as "[llama] sched_reserve:
graph splits = ...". With every layer offloaded (-ngl 99) and every op supported, the graph
has exactly TWO splits: the input embedding's GET_ROWS on the CPU backend (libllama keeps
token_embd in host memory, src/llama-model.cpp:2613) and everything else on MI355X. Any op
this backend's supports_op refuses runs on the CPU as further splits — a silent fallback
that the logits alone do not reveal (mixed K/V cache types did exactly that)."""
import re

UNSPLIT = 2


def graph_splits(stderr):
    """every split count libllama reported (one reserve line per context; "N (with bs=B),
    M (with bs=1)" gives both N and M)"""
    out = []
    for ln in stderr.splitlines():
        if "graph splits" not in ln:
            continue
        rhs = ln.split("graph splits =", 1)[1]
        out += [int(x) for x in re.findall(r"(?<![=\w])(\d+)(?= \(with bs=|\s*$)", rhs.strip())]
    return out


def assert_unsplit(stderr, expected=UNSPLIT):
    s = graph_splits(stderr)
    assert s, "libllama printed no 'graph splits' line (oracle/_ref/ref-llama-bench too old?)"
    assert all(x == expected for x in s), (
        f"graph splits {s}, expected {expected}: some node fell back to the CPU backend\n" +
        "\n".join(ln for ln in stderr.splitlines() if "graph" in ln))

"""CPU tests of the drop-in tests' split-count parser (tests/dropin_util.py): libllama's
scheduler summary lines (src/llama-context.cpp:523-533) in both of their forms."""
import pytest

from dropin_util import assert_unsplit, graph_splits


def test_graph_splits_single_and_dual_forms():
    log = "\n".join([
        "llama_context: n_ctx = 512",
        "[llama] sched_reserve: graph splits = 2",
        "[llama] sched_reserve: graph splits = 3 (with bs=512), 2 (with bs=1)",
        "unrelated line with 7 numbers 8",
    ])
    assert graph_splits(log) == [2, 3, 2]


def test_assert_unsplit_flags_a_fallback():
    assert_unsplit("[llama] sched_reserve: graph splits = 2\n")
    with pytest.raises(AssertionError, match="graph splits"):
        assert_unsplit("[llama] sched_reserve: graph splits = 66 (with bs=512), 2 (with bs=1)\n")
    with pytest.raises(AssertionError, match="no 'graph splits' line"):
        assert_unsplit("llama_context: nothing here\n")

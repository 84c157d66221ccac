"""The reference's own parity harness against this backend: oracle/_ref/test-backend-ops
(tests/test-backend-ops.cpp, compiled unmodified from /root/reference by oracle/Makefile)
in MODE_TEST (:8570-8628) with `-b MI355X0`: every case of each hot-path op family is
evaluated on MI355X0 and on the reference CPU backend and compared with the harness's
own per-op error bounds and sentinels (:1278-1440). A case the backend reports as
unsupported is skipped by the harness (the scheduler would keep it on the CPU); any FAIL
fails the test. Each op (FLASH_ATTN_EXT and MUL_MAT in parameter chunks) is one harness process.
"""
import os
import re
import subprocess
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TBO = os.path.join(ROOT, "oracle", "_ref", "test-backend-ops")
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")
# (op, params regex) chunks, each one harness process of a few seconds to ~1 min
# The harness filters on ggml_op_desc (test-backend-ops.cpp:1249-1275), which names GLU and
# UNARY nodes by their sub-op (ggml.c:1162-1199): "-o GLU" matches nothing. Comma lists are
# one process; SWIGLU_OAI and the UNARY ops the backend reports unsupported are left out so
# every chunk must run > 0 cases.
GLU_OPS = "SWIGLU,GEGLU,REGLU,GEGLU_ERF,GEGLU_QUICK"
UNARY_OPS = ("ABS,SGN,NEG,STEP,TANH,ELU,RELU,SIGMOID,GELU,GELU_QUICK,SILU,HARDSWISH,HARDSIGMOID,EXP,GELU_ERF")
CHUNKS = [(op, None) for op in ["ADD", "MUL", "SCALE", "RMS_NORM", "ROPE", "SOFT_MAX", "SET_ROWS", "GET_ROWS", "CPY",
                                 "CONT", GLU_OPS, UNARY_OPS, "MUL_MAT_ID", "ARGSORT", "SUM_ROWS", "CLAMP", "DIV"]]
CHUNKS += [("MUL_MAT", "type_a=(f32|f16|bf16),"), ("MUL_MAT", "type_a=(q|i|m|t)")]
# the harness's fusion cases (run_whole_graph: the whole graph on the backend, so the
# executor's fusions see these node chains): ROPE -> VIEW -> SET_ROWS (:2377, cases :7082),
# RMS_NORM -> MUL -> ADD and ADD -> RMS_NORM (:3404, :3468, cases :7560-7586), MUL_MAT_ID
# chains (:3920, cases :7790-7831), gate/up GLU GEMVs (:5420, cases :8282-8284) and the
# top-k MoE router (:5322, cases :8297-8304)
CHUNKS += [(op, None) for op in ["ROPE_SET_ROWS", "RMS_NORM_MUL_ADD", "ADD_RMS_NORM", "MUL_MAT_ID_FUSION",
                                 "MUL_MAT_VEC_FUSION", "TOPK_MOE"]]
CHUNKS += [("FLASH_ATTN_EXT", r"hsk=64,"), ("FLASH_ATTN_EXT", r"hsk=128,"), ("FLASH_ATTN_EXT", r"hsk=(40|72|80|96),"),
           ("FLASH_ATTN_EXT", r"hsk=(192|256|576),")]


@pytest.mark.parametrize("op,params", CHUNKS)
def test_reference_harness(tmp_path, op, params):
    if not os.path.exists(TBO):
        pytest.skip("oracle/_ref/test-backend-ops not built")
    env = dict(os.environ, GGML_BACKEND_PATH=LIB)
    cmd = [TBO, "-b", "MI355X0", "-o", op] + (["-p", params] if params else [])
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    log = r.stdout + r.stderr
    fails = [ln for ln in log.splitlines() if "FAIL" in ln]
    assert r.returncode == 0 and not fails, "\n".join(fails[:20]) + log[-3000:]
    m = re.search(r"(\d+)/(\d+) tests passed", log)
    assert m and m.group(1) == m.group(2) and int(m.group(2)) > 0, log[-2000:]
    assert re.search(r"Backend MI355X0:.*OK", log), log[-2000:]
    n_uns = log.count("not supported")
    print(f"{op[:40]} {params or ''}: {m.group(1)} passed, {n_uns} not supported, {time.time() - t0:.0f} s")

#!/usr/bin/env python3
"""Diagnostic: where does the 70B-width pp512 logits error come from? Runs the reference
libllama on the llama3_70b_2l GGUF at -ngl 0 (reference CPU backend) and -ngl 99 (this
backend) under several executor settings and prints per-position NMSE of the 16 last
positions, the GPU-vs-GPU NMSE between settings, and the 8B-width figure beside it."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
REF = os.path.join(ROOT, "oracle", "_ref", "ref-llama-bench")
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")


def nmse(a, b):
    a = a.astype(np.float64); b = b.astype(np.float64)
    return float(np.sum((a - b) ** 2) / max(np.sum(b ** 2), 1e-30))


def run(d, gguf, toks, ngl, fa, env_extra=None, tag=""):
    tf, of = os.path.join(d, "t.i32"), os.path.join(d, f"o{ngl}{fa}{tag}.f32")
    np.asarray(toks, np.int32).tofile(tf)
    env = dict(os.environ)
    if ngl:
        env["GGML_BACKEND_PATH"] = LIB
    env.update(env_extra or {})
    r = subprocess.run([REF, "-m", gguf, "-t", "16", "-ngl", str(ngl), "-fa", str(fa), "--logits", tf, of, "--last", "16"],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    nv = int(r.stdout.split('"n_vocab": ')[1].split("}")[0])
    return np.fromfile(of, np.float32).reshape(-1, nv)


def main():
    d = tempfile.mkdtemp()
    for shape in ("llama3_70b_2l", "llama3_8b_2l"):
        g = os.path.join(d, shape + ".gguf")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gguf_synth.py"), "--shape", shape, "--recipe", "q4_k_m",
                        "--out", g], check=True, stdout=subprocess.DEVNULL)
        toks = np.random.default_rng(32).integers(0, 128000, 512)
        for fa in (1, 0):
            cpu = run(d, g, toks, 0, fa)
            arms = {"default": {}, "mmq4_off": {"GGML_MI355X_MMQ4_OFF": "1"}, "no_fusion": {"GGML_MI355X_DISABLE_FUSION": "1"}}
            outs = {k: run(d, g, toks, 99, fa, v, k) for k, v in arms.items()}
            for k, o in outs.items():
                per = [nmse(o[i], cpu[i]) for i in range(len(o))]
                print(f"{shape} fa{fa} {k:10s} vs cpu nmse {nmse(o, cpu):.3e}  per-pos min {min(per):.2e} max {max(per):.2e}  "
                      f"top1 {np.mean(o.argmax(1) == cpu.argmax(1)):.2f}", flush=True)
            print(f"{shape} fa{fa} default vs mmq4_off {nmse(outs['default'], outs['mmq4_off']):.3e}  "
                  f"default vs no_fusion {nmse(outs['default'], outs['no_fusion']):.3e}", flush=True)
        os.remove(g)


if __name__ == "__main__":
    main()

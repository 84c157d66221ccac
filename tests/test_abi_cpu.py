"""CPU checks of the drop-in boundary: the C-ABI library loads without a GPU and
exports every entry point the public headers declare (include/*.h), and the struct
layouts in include/ggml_abi.h match the reference's ggml.h when it is present."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "llama-mi50.cpp_amd", "lib", "libggml-mi355x.so")
HEADERS = ["ggml_mi355x.h", "mx_graph.h", "mx_llama.h"]


def declared_functions(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set()
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src):
        name = m.group(1)
        if name.startswith(("ggml_backend_", "mxg_", "mxr_")) and not name.endswith("_t"):
            names.add(name)
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


@pytest.fixture(scope="module")
def lib_built():
    if not os.path.exists(LIB):
        pytest.skip("library not built (run __graft_entry__.build())")
    return LIB


@pytest.mark.parametrize("header", HEADERS)
def test_header_symbols_exported(lib_built, header):
    decl = declared_functions(header)
    assert decl, f"no declarations parsed from {header}"
    missing = decl - exported_symbols()
    assert not missing, f"{header}: not exported: {sorted(missing)}"


def test_ggml_backend_entry_points(lib_built):
    # the two symbols ggml-backend-reg.cpp:219-231 dlsym()s
    syms = exported_symbols()
    assert "ggml_backend_init" in syms and "ggml_backend_score" in syms


def test_library_loads_without_gpu(lib_built):
    lib = ctypes.CDLL(lib_built)
    lib.ggml_backend_score.restype = ctypes.c_int
    # score may be 0 here (no device); the call must not crash
    assert lib.ggml_backend_score() >= 0


def test_abi_layout_matches_reference(tmp_path):
    """Compile a probe that includes BOTH the reference ggml.h and our ABI mirror in
    separate translation units and compares sizeof/offsetof. Skipped on the GPU box."""
    ref_inc = "/root/reference/ggml/include"
    if not os.path.isdir(ref_inc):
        pytest.skip("reference headers not present")
    fields = ["ne", "nb", "op", "op_params", "flags", "src", "view_src", "view_offs", "data", "name", "extra"]
    probe = lambda inc, hdr: "\n".join([
        f'#include "{hdr}"', "#include <stddef.h>", "#include <stdio.h>",
        "void dump(FILE*f){",
        'fprintf(f,"tensor %zu\\n",sizeof(struct ggml_tensor));',
        *[f'fprintf(f,"{x} %zu\\n",offsetof(struct ggml_tensor,{x}));' for x in fields],
        'fprintf(f,"op_fa %d unary %d glu %d count %d\\n",(int)GGML_OP_FLASH_ATTN_EXT,(int)GGML_OP_UNARY,(int)GGML_OP_GLU,(int)GGML_OP_COUNT);',
        'fprintf(f,"types %d\\n",(int)GGML_TYPE_COUNT);',
        "}", "int main(){dump(stdout);return 0;}"])
    outs = []
    for inc, hdr in [(ref_inc, "ggml.h"), (os.path.join(ROOT, "include"), "ggml_abi.h")]:
        c = tmp_path / f"p_{hdr}.c"
        c.write_text(probe(inc, hdr))
        exe = tmp_path / f"p_{hdr}"
        subprocess.run(["gcc", "-std=gnu11", "-I", inc, str(c), "-o", str(exe)], check=True)
        outs.append(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    assert outs[0] == outs[1]


# the backend vtables and the structs that embed them (ggml/src/ggml-backend-impl.h:17-210,
# ggml/include/ggml-backend.h:140-170 for the device props/caps): member order, offsets
# and sizes of include/ggml_abi.h against the reference headers
VTABLE_STRUCTS = ["ggml_backend_buffer_type_i", "ggml_backend_buffer_type", "ggml_backend_buffer_i",
                  "ggml_backend_buffer", "ggml_backend_i", "ggml_backend", "ggml_backend_event",
                  "ggml_backend_device_i", "ggml_backend_device", "ggml_backend_reg_i", "ggml_backend_reg",
                  "ggml_backend_dev_caps", "ggml_backend_dev_props", "ggml_backend_feature"]


def struct_members(src, name):
    m = re.search(r"struct\s+" + name + r"\s*\{(.*?)\n\s*\};", src, flags=re.S)
    assert m, f"struct {name} not found in include/ggml_abi.h"
    body = re.sub(r"//[^\n]*", "", m.group(1))
    members = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        fp = re.search(r"\(\s*\*\s*(\w+)\s*\)", decl)
        members.append(fp.group(1) if fp else re.findall(r"(\w+)\s*(?:\[[^\]]*\])?\s*$", decl)[0])
    return members


def test_vtable_layout_matches_reference(tmp_path):
    """sizeof / offsetof of every backend vtable member: a reordered or missing function
    pointer would make libllama call the wrong entry point. Skipped on the GPU box."""
    ref_root = "/root/reference/ggml"
    if not os.path.isdir(ref_root):
        pytest.skip("reference headers not present")
    src = open(os.path.join(ROOT, "include", "ggml_abi.h")).read()
    lines = []
    for s in VTABLE_STRUCTS:
        mem = struct_members(src, s)
        assert mem, s
        lines.append(f'fprintf(f,"{s} %zu\\n",sizeof(struct {s}));')
        lines += [f'fprintf(f,"{s}.{x} %zu\\n",offsetof(struct {s},{x}));' for x in mem]
    probe = lambda hdr: "\n".join([f'#include "{hdr}"', "#include <stddef.h>", "#include <stdio.h>",
                                   "void dump(FILE*f){", *lines, "}", "int main(){dump(stdout);return 0;}"])
    outs = []
    for incs, hdr in [([f"{ref_root}/include", f"{ref_root}/src"], "ggml-backend-impl.h"),
                      ([os.path.join(ROOT, "include")], "ggml_abi.h")]:
        c = tmp_path / f"v_{hdr}.c"
        c.write_text(probe(hdr))
        exe = tmp_path / f"v_{hdr}"
        args = ["gcc", "-std=gnu11"] + [a for i in incs for a in ("-I", i)] + [str(c), "-o", str(exe)]
        subprocess.run(args, check=True)
        outs.append(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    assert outs[0].count("\n") > 80
    assert outs[0] == outs[1]

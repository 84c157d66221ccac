"""llama-mi50.cpp_amd — MI355X-native ggml backend (libggml-mi355x.so) plus the
host-side mirror of the reference's graph API used by tests and the bench.

The directory name is not a Python identifier; import it with ``load_package()``
from the repo root helpers (tests/conftest.py, bench.py, __graft_entry__.py).
"""
from . import _lib  # noqa: F401
from .ggml import Backend, Context, Tensor, row_bytes  # noqa: F401
from .llama import Model, Session, LLAMA3_8B, LLAMA3_70B, TINYLLAMA_1B, MIXTRAL_8X7B  # noqa: F401

LIB_PATH = _lib.LIB_PATH


def device_count():
    """MI355X devices the backend sees (initialises HIP)."""
    return int(_lib.load().ggml_backend_mi355x_get_device_count())

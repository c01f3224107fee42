"""The C-ABI library loads on a CPU-only host and exports every symbol include/chiara.h
declares (no compute calls without a GPU)."""
import os
import re
import shutil
import subprocess

import pytest

import chiara_amd as ca
from chiara_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(REPO, "include", "chiara.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(chr_[a-z_]+)\s*\(", hdr)))


def test_header_symbols_exported():
    decl = _declared()
    assert len(decl) >= 20
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r"\bT (chr_\w+)", out))
    missing = [s for s in decl if s not in exported]
    assert not missing, f"declared but not exported: {missing}"
    assert sorted(_lib.EXPORTED) == decl


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded HIP fat binary targets gfx950


def test_abi_basics():
    assert ca.lib().chr_abi_version() == 11
    assert ca.lib().chr_error_string(2).decode().startswith("count")
    assert ca.lib().chr_error_string(0) == b"success"


def test_no_cpu_fallback_for_compute():
    """Without a device the compute entry points fail with an error code (no CPU path)."""
    import torch

    if torch.cuda.is_available():
        return
    g = ca.lib().chr_local_group_create
    import ctypes

    h = ctypes.c_void_p()
    assert g(ctypes.byref(h), 2, 0) == 6  # CHR_ERR_NO_DEVICE


def test_profile_phases_rejects_null_comm():
    assert ca.lib().chr_comm_profile_phases(None, None, 0, 0) == -1


def test_reduce_tree_rejects_bad_args_without_device():
    import ctypes

    leaves = (ctypes.c_void_p * 2)(0x1000, 0x2000)
    assert ca.lib().chr_reduce_tree(0x3000, leaves, 2, bytes([0, 1]), None, 0, 11, ca.SUM, None) == 1  # bad dtype
    assert ca.lib().chr_reduce_tree(0x3000, None, 2, bytes([0, 1]), None, 0, ca.FLOAT32, ca.SUM, None) == 1


def _ipc_env_after_dlopen(preset):
    """Loads libchiara.so into a fresh process (no torch, no chiara_amd) and reads the C-level
    environment afterwards."""
    code = (
        "import ctypes, sys\n"
        f"ctypes.CDLL({_lib.LIB_PATH!r})\n"
        "libc = ctypes.CDLL(None)\n"
        "libc.getenv.restype = ctypes.c_char_p\n"
        "v = libc.getenv(b'HSA_ENABLE_IPC_MODE_LEGACY')\n"
        "print(v.decode() if v is not None else 'UNSET')\n"
    )
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    if preset is not None:
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = preset
    return subprocess.check_output(["python3", "-c", code], env=env).decode().strip()


def test_library_leaves_the_environment_alone():
    """loading the library changes no process-wide setting (the entry paths set it)."""
    assert _ipc_env_after_dlopen(None) == "UNSET"
    assert _ipc_env_after_dlopen("1") == "1"


def test_shim_entry_path_defaults_ipc_mode(tmp_path):
    """The MPI shim, linked into a reference harness executable, sets the dmabuf-IPC default at program
    load (before main, MPI_Init and any HIP call); a caller's value is kept.  Built here from the shim
    and a two-line main, with the package Makefile's harness flags."""
    import shutil

    mpi_home = "/opt/conda"
    if not os.path.exists(os.path.join(mpi_home, "include", "mpi.h")) or not shutil.which("g++"):
        pytest.skip("MPICH headers or g++ absent")
    pkg = _lib.PKG_ROOT
    src = tmp_path / "probe.cpp"
    src.write_text('#include <cstdio>\n#include <cstdlib>\nint main() { const char* v = '
                   'std::getenv("HSA_ENABLE_IPC_MODE_LEGACY"); std::printf("%s\\n", v ? v : "UNSET"); }\n')
    exe = tmp_path / "probe"
    subprocess.check_call(["g++", "-O1", "-std=c++17", f"-I{REPO}/include", "-I/opt/rocm/include",
                           f"-I{mpi_home}/include", "-D__HIP_PLATFORM_AMD__", "-o", str(exe), str(src),
                           os.path.join(pkg, "csrc", "shim", "chiara_mpi_shim.cpp"),
                           f"-L{os.path.dirname(_lib.LIB_PATH)}", "-lchiara", "-L/opt/rocm/lib", "-lamdhip64",
                           f"{mpi_home}/lib/libmpi.so", f"-Wl,-rpath,{os.path.dirname(_lib.LIB_PATH)}",
                           "-Wl,-rpath,/usr/lib/x86_64-linux-gnu", "-Wl,-rpath,/opt/rocm/lib",
                           f"-Wl,-rpath,{mpi_home}/lib"])
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    assert subprocess.check_output([str(exe)], env=env).decode().strip() == "0"
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "1"
    assert subprocess.check_output([str(exe)], env=env).decode().strip() == "1"


def test_package_defaults_ipc_mode_before_torch():
    code = "import os, chiara_amd; print(os.environ['HSA_ENABLE_IPC_MODE_LEGACY'])"
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    env["PYTHONPATH"] = _lib.PKG_ROOT + os.pathsep + env.get("PYTHONPATH", "")
    out = subprocess.check_output(["python3", "-c", code], env=env, cwd=REPO).decode().strip()
    assert out == "0"


def test_user_op_registry_on_the_host():
    """chr_op_create / chr_op_free (ABI 11) need no GPU: codes from 64 up, a NULL launcher refused, a freed code
    reusable and refused once freed, and every slot taken after 64 live ops."""
    import ctypes

    L = ca.lib()
    fn = ctypes.cast(L.chr_abi_version, ctypes.c_void_p).value  # any address: never called here
    op = ctypes.c_int(-1)
    assert L.chr_op_create(None, None, 0, ctypes.byref(op)) == ca.ERR_INVALID_ARG
    made = []
    for _ in range(64):
        assert L.chr_op_create(fn, None, 0, ctypes.byref(op)) == 0
        made.append(op.value)
    assert sorted(made) == list(range(64, 128))
    assert L.chr_op_create(fn, None, 1, ctypes.byref(op)) == ca.ERR_UNSUPPORTED
    assert L.chr_op_free(made[5]) == 0 and L.chr_op_free(made[5]) == ca.ERR_INVALID_ARG
    assert L.chr_op_create(fn, None, 1, ctypes.byref(op)) == 0 and op.value == made[5]
    for o in made:
        assert L.chr_op_free(o) == 0
    assert L.chr_op_free(3) == ca.ERR_INVALID_ARG and L.chr_op_free(200) == ca.ERR_INVALID_ARG


def test_shim_exports_the_user_op_binding():
    """The MPI-signature shim (linked into the harness executables) defines chiara_shim_op_bind / _unbind: a user
    MPI_Op gets its device twin there (csrc/shim/chiara_mpi_shim.cpp); exercised under mpiexec by
    test_gpu_ref_harness.py::test_shim_over_mpi_datatype_op_table."""
    exe = os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd", "bin", "chiara_shim_types")
    if not os.path.exists(exe) or not shutil.which("nm"):
        pytest.skip("shim harness not built here")
    syms = subprocess.check_output(["nm", "-C", exe]).decode()
    for name in ("chiara_shim_op_bind", "chiara_shim_op_unbind", "all_reduce_radix_batch(char*"):
        assert f" T {name}" in syms, name

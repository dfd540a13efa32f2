"""Build of the host helper extension (csrc/nfk_host.cpp -> _nfk_host*.so, in
tree next to libnfk.so): g++ against the installed torch's headers and
libraries.  Called by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))


def target():
    return os.path.join(HERE, "_nfk_host" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force=False):
    import torch
    import torch.utils.cpp_extension as ce
    src = os.path.join(HERE, "csrc", "nfk_host.cpp")
    out = target()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    inc = ce.include_paths() + [sysconfig.get_paths()["include"]]
    lib = ce.library_paths()[0]
    abi = "1" if torch._C._GLIBCXX_USE_CXX11_ABI else "0"
    cmd = (["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-D_GLIBCXX_USE_CXX11_ABI=" + abi, src, "-o", out]
           + ["-I" + p for p in inc] + ["-L" + lib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
                                        "-Wl,-rpath," + lib])
    subprocess.run(cmd, check=True)
    return out

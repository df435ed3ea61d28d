"""Build the gfx950 engine library in-tree: anothertls_amd/libatls.so (hipcc, no torch)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libatls.so")
SOURCES = ["engine.cpp", "keysetup.hip", "plan.hip", "gcm.hip", "chacha.hip", "hkdf.hip", "aes_block.hip", "diag.hip", "stream.cpp", "multi.cpp"]
ARCH = os.environ.get("ATLS_OFFLOAD_ARCH", "gfx950")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    # sources only: variant builds write objects under csrc/_obj, which must not make this look stale
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h"))]
    deps.append(os.path.join(HERE, "..", "include", "atls.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, defines=(), out=None, flags=()):
    """defines: extra -D flags (kernel tuning variants); flags: extra compiler flags (variant builds only);
    out: alternate library path."""
    lib = out or LIB
    if not force and not defines and not flags and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmds, objs = [], []
    for src in SOURCES:
        tag = "_".join([d.replace("=", "") for d in defines] + [str(abs(hash(flags)) % 10**8)] * bool(flags))
        obj = os.path.join(CSRC, "_obj", (tag + "_" if tag else "") + src + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "hip"]
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result",
               "-munsafe-fp-atomics", *flags, *[f"-D{d}" for d in defines], *lang, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(obj)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(cmds), os.cpu_count() or 1, 8)) as pool:
        list(pool.map(subprocess.check_call, cmds))
    os.makedirs(os.path.dirname(os.path.abspath(lib)), exist_ok=True)
    tmp = lib + ".tmp"
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs])
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))

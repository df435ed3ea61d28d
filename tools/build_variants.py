"""Build library variants for same-box A/Bs: python tools/build_variants.py name=DEF1,DEF2,+-flag name2= ...
Each becomes anothertls_amd/variants/libatls_<name>.so (an empty define list = the default build)."""
import importlib.util
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("b", os.path.join(ROOT, "anothertls_amd", "_build.py"))
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
vdir = os.path.join(ROOT, "anothertls_amd", "variants")
if "--clean" in sys.argv:
    shutil.rmtree(vdir, ignore_errors=True)
for arg in sys.argv[1:]:
    if arg.startswith("--"):
        continue
    name, _, defs = arg.partition("=")
    # a list item starting with '+' is a raw compiler flag ('+-mllvm +-amdgpu-sched-strategy=max-ilp')
    defines = tuple(d for d in defs.split(",") if d and not d.startswith("+"))
    flags = tuple(d[1:] for d in defs.split(",") if d.startswith("+"))
    out = os.path.join(vdir, f"libatls_{name}.so")
    b.build(force=True, defines=defines or ("ATLS_VARIANT_" + name,), out=out, flags=flags)
    print(out, defines, flags)

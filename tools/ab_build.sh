#!/bin/bash
# Build anothertls_amd/variants/libatls_<name>.so from a git revision (default HEAD) of csrc/,
# for same-box A/B timing: bash tools/ab_build.sh <name> [rev]
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:-HEAD}
tmp=$(mktemp -d)
git archive "$rev" anothertls_amd include | tar -x -C "$tmp"
python3 - "$tmp" "$name" <<'PY'
import importlib.util, os, sys
tmp, name = sys.argv[1], sys.argv[2]
spec = importlib.util.spec_from_file_location("b", os.path.join(tmp, "anothertls_amd", "_build.py"))
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
out = os.path.abspath(os.path.join("anothertls_amd", "variants", f"libatls_{name}.so"))
os.makedirs(os.path.dirname(out), exist_ok=True)
b.build(force=True, out=out)
print(out)
PY
rm -rf "$tmp"

export LENS=1008,16368
for v in libatls.so variants/libatls_dbg8.so variants/libatls_dbg16.so variants/libatls_dbg2.so; do
  echo "== $v"; ATLS_LIB=$PWD/anothertls_amd/$v timeout -k 10 120 python tools/len_sweep.py 2>&1 | grep -v amdgpu.ids || exit 1
done

# Measurement variants of libbra_hip.so (each with one -D knob), built in-tree under build/variants/.
# usage: bash scripts/build_variants.sh NAME:FLAGS ...   e.g. nosort:-DBRA_EXP_NOSORT
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=br-archive_amd/build/variants/$name
  mkdir -p $out && rm -f $out/libbra_hip.so $out/*.o
  make -C br-archive_amd -s OBJDIR=$PWD/$out/obj EXTRA="$flags" $PWD/$out/libbra_hip.so HERE=$PWD/br-archive_amd/ >/dev/null 2>&1 || \
    (for f in bwt bwt_large mtf rle rle_decode huffman ibwt crc capi selftest; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result $flags -c br-archive_amd/csrc/$f.hip -o $out/$f.o & done; wait; /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libbra_hip.so $out/*.o)
  echo "built $out/libbra_hip.so ($flags)"
done

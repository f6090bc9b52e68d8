#!/bin/bash
# Build ab/lib<name>.so: the in-tree objects with csrc/<file>.hip recompiled under extra defines
# (diagnostic / A-B variants).  usage: bash tools/variant_lib.sh <name> <file-stem> -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1 stem=$2; shift 2
P=eeg-multimodal_amd
python -c "import sys; sys.path.insert(0,'$P'); from eegfusion.build import build; build()" > /dev/null
mkdir -p ab /tmp/vlib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Wno-unused-result \
  -Wno-inline-asm -Iinclude -I$P/csrc "$@" -c $P/csrc/$stem.hip -o /tmp/vlib/$name.$stem.o
objs=$(ls $P/build/*.o | grep -v "/$stem.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/lib$name.so $objs /tmp/vlib/$name.$stem.o
echo ab/lib$name.so

#!/bin/bash
# Link an A/B variant of libvit_hip.so: the in-tree objects with csrc/$1 taken from git revision $2
# (default HEAD) -> vit-of-pytorch_amd/vitmi/ab/libvit_hip.so; time it with VITMI_LIB=<that path>.
set -e
SRC=$1; REV=${2:-HEAD}
cd "$(dirname "$0")/../vit-of-pytorch_amd"
mkdir -p build/ab vitmi/ab
git show "$REV:./csrc/$SRC" > build/ab/$SRC
cp csrc/*.h csrc/*.inc build/ab/ 2>/dev/null || true
EXTRA=""
case $SRC in attention*.hip) EXTRA="-mno-amdgpu-ieee -fno-honor-nans -fno-strict-aliasing";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -mcode-object-version=5 $EXTRA -I csrc -c build/ab/$SRC -o build/ab/${SRC%.hip}.o
OBJS=$(ls build/*.o | grep -v "build/${SRC%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build/ab/${SRC%.hip}.o -o vitmi/ab/libvit_hip.so
echo "vitmi/ab/libvit_hip.so: $SRC from $REV"

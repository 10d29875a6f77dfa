#!/bin/bash
# usage: scripts/mkvar_obj.sh NAME SRC [hipcc flags] -> variants/NAME/liblfm.so with csrc/SRC.hip rebuilt with the flags
set -e
cd /root/repo/lightfieldmicroscopy_pc-bzip2_amd
name=$1; src=$2; shift 2
mkdir -p /tmp/vb/$name /root/repo/variants/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include/lfm -Icsrc --offload-arch=gfx950 -munsafe-fp-atomics "$@" -c csrc/$src.hip -o /tmp/vb/$name/$src.o 2>&1 | { grep -E " error" -A3 || true; }
test -f /tmp/vb/$name/$src.o
/opt/rocm/bin/hipcc -shared -fPIC -o /root/repo/variants/$name/liblfm.so $(ls build/*.o | grep -v "/$src.o") /tmp/vb/$name/$src.o -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -l:libbz2.so.1.0 -lz -lpthread -Wl,-rpath,/opt/rocm/lib
echo built $name

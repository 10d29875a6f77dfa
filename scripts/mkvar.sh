#!/bin/bash
# usage: mkvar.sh NAME [extra hipcc flags]  -> /root/repo/variants/NAME/liblfm.so (lfm_bzip2.hip rebuilt with flags)
set -e
cd /root/repo/lightfieldmicroscopy_pc-bzip2_amd
name=$1; shift
rm -f /tmp/vb/$name/lfm_bzip2.o; mkdir -p /tmp/vb/$name /root/repo/variants/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include/lfm -Icsrc --offload-arch=gfx950 -munsafe-fp-atomics "$@" -c csrc/lfm_bzip2.hip -o /tmp/vb/$name/lfm_bzip2.o 2>&1 | { grep -E "error" -A3 || true; }; test -f /tmp/vb/$name/lfm_bzip2.o
/opt/rocm/bin/hipcc -shared -fPIC -o /root/repo/variants/$name/liblfm.so $(ls build/*.o | grep -v lfm_bzip2.o) /tmp/vb/$name/lfm_bzip2.o -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -l:libbz2.so.1.0 -lz -lpthread -Wl,-rpath,/opt/rocm/lib
echo built $name

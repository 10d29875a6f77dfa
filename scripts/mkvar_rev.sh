#!/bin/bash
# usage: scripts/mkvar_rev.sh NAME REV -> variants/NAME/liblfm.so with lfm_bzip2.hip from git revision REV
set -e
cd /root/repo/lightfieldmicroscopy_pc-bzip2_amd
name=$1; rev=$2
mkdir -p /tmp/vb/$name /root/repo/variants/$name
git show $rev:lightfieldmicroscopy_pc-bzip2_amd/csrc/lfm_bzip2.hip > csrc/_rev_bzip2.hip
trap 'rm -f csrc/_rev_bzip2.hip' EXIT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include/lfm -Icsrc --offload-arch=gfx950 -munsafe-fp-atomics -c csrc/_rev_bzip2.hip -o /tmp/vb/$name/lfm_bzip2.o 2>&1 | { grep -E " error" -A3 || true; }
/opt/rocm/bin/hipcc -shared -fPIC -o /root/repo/variants/$name/liblfm.so $(ls build/*.o | grep -v lfm_bzip2.o) /tmp/vb/$name/lfm_bzip2.o -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -l:libbz2.so.1.0 -lz -lpthread -Wl,-rpath,/opt/rocm/lib
echo built $name from $rev

// bz2_sys.h -- the two libbz2 entry points liblfm uses (public bzlib API,
// stable since bzip2 1.0).  The image ships libbz2.so.1.0 without its
// development header, so the prototypes are declared here; liblfm links the
// system library, whose output is byte-identical to the reference's vendored
// 1.0.6 on the reference's own known-answer tests (tests/test_oracle.py).
#pragma once
extern "C" {
int BZ2_bzBuffToBuffCompress(char* dest, unsigned int* destLen, char* source, unsigned int sourceLen,
                             int blockSize100k, int verbosity, int workFactor);
int BZ2_bzBuffToBuffDecompress(char* dest, unsigned int* destLen, char* source, unsigned int sourceLen, int small,
                               int verbosity);
}
#define LFM_BZ_OK 0

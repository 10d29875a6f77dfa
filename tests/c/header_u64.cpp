// klb_image_header with end-offsets past 2^32 (TEST INFRASTRUCTURE): the
// reference stores u64 blockOffset (src/klb_imageHeader.h:46, written by
// klb_imageIO.cpp:1215-1217).  A 100-volume config-5 stack (51.6 GB .lfm)
// needs them.  The header is written with writeHeader(FILE*) through
// liblfm.so and read back with readHeader(path), parseHeader(buf) and the C
// ABI readKLBheader; the bytes go to stdout as hex for the Python test to
// compare with the reference's own class (oracle/_ref/libklbheader_ref.so).
// usage: header_u64 PATH
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include "klb_Cwrapper.h"
#include "klb_imageHeader.h"

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    const uint32_t xyzct[5] = {4096, 4096, 32, 1, 100};
    const uint32_t bs[5] = {96, 96, 8, 1, 1};
    const float ps[5] = {1, 1, 2.5f, 1, 1};
    char md[KLB_METADATA_SIZE] = "u64 offsets";
    klb_image_header h;
    h.setHeader(xyzct, UINT16_TYPE, ps, bs, BZIP2, md, 0x80 | 4, 13);
    const size_t nb = h.calculateNumBlocks();
    if (nb != 43u * 43u * 4u * 100u) return 3;
    h.resizeBlockOffset(nb);
    // cumulative end-offsets of ~70 kB blocks: past 2^32 after ~61 000 blocks
    uint64_t acc = 0;
    for (size_t i = 0; i < nb; ++i) {
        acc += 70000 + (i * 7919) % 5003;
        h.blockOffset[i] = acc;
    }
    if (h.blockOffset[nb - 1] <= (1ull << 32)) return 4;
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) return 5;
    h.writeHeader(f);
    std::fclose(f);
    int bad = 0;
    klb_image_header r;
    if (r.readHeader(argv[1]) != 0) return 6;
    std::vector<unsigned char> buf(h.getSizeInBytes());
    f = std::fopen(argv[1], "rb");
    if (!f || std::fread(buf.data(), 1, buf.size(), f) != buf.size()) return 7;
    std::fclose(f);
    klb_image_header p;
    if (p.parseHeader(buf.data(), buf.size()) != 0) return 8;
    for (const klb_image_header* x : {&r, &p}) {
        if (x->getNumBlocks() != nb || x->headerVersion != (0x80 | 4) || x->Nnum != 13) ++bad;
        for (size_t i = 0; i < nb; ++i)
            if (x->getBlockOffset(i) != (i ? h.blockOffset[i - 1] : 0) ||
                x->getBlockCompressedSizeBytes(i) != h.blockOffset[i] - (i ? h.blockOffset[i - 1] : 0))
                ++bad;
        if (x->getCompressedFileSizeInBytes() != h.getSizeInBytes() + h.blockOffset[nb - 1]) ++bad;  // (header included, klb_imageHeader.cpp:256-259)
    }
    uint32_t rx[5], rbs[5];
    float rps[5];
    KLB_DATA_TYPE dt;
    KLB_COMPRESSION_TYPE ct;
    char rmd[KLB_METADATA_SIZE];
    if (readKLBheader(argv[1], rx, &dt, rps, rbs, &ct, rmd) != 0 || std::memcmp(rx, xyzct, sizeof(rx)) ||
        std::memcmp(rbs, bs, sizeof(rbs)) || dt != UINT16_TYPE || ct != BZIP2)
        ++bad;
    std::printf("last_offset %llu bad %d\n", (unsigned long long)h.blockOffset[nb - 1], bad);
    return bad ? 1 : 0;
}

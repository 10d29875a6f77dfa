// boundary_main.cpp -- a C/C++ caller of the drop-in boundary, linked
// against liblfm.so the way the reference's callers link (TEST
// INFRASTRUCTURE, driven by tests/test_boundary_gpu.py).
//
//   boundary_main <input.u16> X Y Z <outdir> <predictor_request> <video>
//
// 1. writeKLBstack on the uint16 stack (auto-select, Nnum 13:
//    reference src/klb_Cwrapper.cpp:19-50) -> outdir/klb.lfm
// 2. readKLBstack (malloc'ed result, freed by the caller, :112-151) and
//    readKLBstackInPlace (:154) -> every pixel compared with the input
// 3. the MEX writeLFMstack member sequence on klb_imageIO
//    (matlabWrapper/writeLFMstack.cpp:56-448: setHeader fields,
//    header.setDefaultBlockSize(), headerVersion |= request, Nnum,
//    headerVersion |= video << 7, writeImage) -> outdir/mex.lfm, then the
//    readLFMstack sequence (readLFMstack.cpp:61-133: readHeader,
//    readImageFull) -> compared with the input
// 4. readKLBroiInPlace of a corner ROI -> compared with the crop
// 5. readKLBheader fields
// 6. the public selection helpers of klb_imageIO (src/klb_imageIO.h:91,101):
//    bwt_entropy_2D on a device copy of frame 0 -- candidate 0 (is_src 0) is
//    reported as (float)(e * 0.96) with 0.96 a double (klb_imageIO.cpp:2090);
//    predict_and_2DEntropy over the 8 candidates
// Prints one line per check; exit 0 only if every check passed.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "klb_Cwrapper.h"
#include "klb_imageIO.h"
#include "lfm_api.h"
#include "lfm_hip.h"

// HIP runtime entry points (C linkage in libamdhip64) for the device buffers
// the selection helpers take; declared here so this caller builds with g++
extern "C" int hipMalloc(void** p, size_t n);
extern "C" int hipMemcpy(void* dst, const void* src, size_t n, int kind);
extern "C" int hipFree(void* p);

static int failures = 0;
static void check(bool ok, const char* what)
{
    std::printf("%s %s\n", ok ? "OK  " : "FAIL", what);
    if (!ok) ++failures;
}

int main(int argc, char** argv)
{
    // line-buffered: a caller that kills this program still sees every check
    // printed before the kill (stdout is a pipe under the tests)
    std::setvbuf(stdout, nullptr, _IOLBF, 0);
    if (argc != 8) {
        std::fprintf(stderr, "usage: %s input.u16 X Y Z outdir request video\n", argv[0]);
        return 2;
    }
    const uint32_t X = (uint32_t)std::atoi(argv[2]), Y = (uint32_t)std::atoi(argv[3]), Z = (uint32_t)std::atoi(argv[4]);
    const std::string out = argv[5];
    const int request = std::atoi(argv[6]), video = std::atoi(argv[7]);
    const size_t n = (size_t)X * Y * Z;
    std::vector<uint16_t> img(n);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f || std::fread(img.data(), 2, n, f) != n) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    std::fclose(f);

    // 1. writeKLBstack: headerVersion 0 (auto-select), Nnum 13, default blocks
    const std::string klb = out + "/klb.lfm";
    uint32_t xyzct[KLB_DATA_DIMS] = {X, Y, Z, 1, 1};
    float32_t ps[KLB_DATA_DIMS] = {1.f, 1.f, 1.f, 1.f, 1.f};
    char meta[KLB_METADATA_SIZE] = "boundary_main";
    check(writeKLBstack(img.data(), klb.c_str(), xyzct, UINT16_TYPE, -1, ps, nullptr, BZIP2, meta) == 0,
          "writeKLBstack uint16 auto-select");

    // 2. readKLBstack (caller frees) and readKLBstackInPlace
    {
        uint32_t rx[KLB_DATA_DIMS], rb[KLB_DATA_DIMS];
        float32_t rps[KLB_DATA_DIMS];
        KLB_DATA_TYPE dt;
        KLB_COMPRESSION_TYPE ct;
        char rmeta[KLB_METADATA_SIZE];
        void* p = readKLBstack(klb.c_str(), rx, &dt, -1, rps, rb, &ct, rmeta);
        check(p != nullptr, "readKLBstack returns a buffer");
        if (p) {
            check(std::memcmp(p, img.data(), n * 2) == 0, "readKLBstack pixels equal the input");
            check(rx[0] == X && rx[1] == Y && rx[2] == Z && dt == UINT16_TYPE && ct == BZIP2,
                  "readKLBstack dims / type / compression");
            check(std::strcmp(rmeta, "boundary_main") == 0, "readKLBstack metadata");
            std::free(p);
        }
        std::vector<uint16_t> back(n, 0xABCD);
        KLB_DATA_TYPE dt2;
        check(readKLBstackInPlace(klb.c_str(), back.data(), &dt2, -1) == 0 && dt2 == UINT16_TYPE,
              "readKLBstackInPlace rc 0");
        check(back == img, "readKLBstackInPlace pixels equal the input");
    }

    // 3. the MEX writeLFMstack / readLFMstack member sequence
    const std::string mex = out + "/mex.lfm";
    {
        klb_imageIO io(mex);
        for (int d = 0; d < KLB_DATA_DIMS; ++d) {
            io.header.xyzct[d] = xyzct[d];
            io.header.pixelSize[d] = ps[d];
        }
        io.header.dataType = UINT16_TYPE;
        io.header.compressionType = BZIP2;
        io.header.setDefaultBlockSize();
        io.header.headerVersion = 0;
        io.header.headerVersion |= (uint8_t)request;
        io.header.Nnum = 13;
        io.header.headerVersion |= (uint8_t)(video << 7);
        check(io.writeImage((const char*)img.data(), -1) == 0, "klb_imageIO::writeImage (MEX sequence)");

        klb_imageIO rd(mex);
        check(rd.readHeader() == 0, "klb_imageIO::readHeader");
        check(rd.header.xyzct[2] == Z && rd.header.Nnum == 13 && (rd.header.headerVersion >> 7) == video,
              "header fields (dims, Nnum, video bit)");
        std::vector<uint16_t> back(rd.header.getImageSizePixels());
        check(rd.readImageFull((char*)back.data(), -1) == 0 && back == img, "klb_imageIO::readImageFull pixels");
        std::printf("INFO mex headerVersion %d\n", (int)rd.header.headerVersion);
    }

    // 4. ROI read of the lower-right corner (needs every block up / left of it)
    {
        uint32_t lb[KLB_DATA_DIMS] = {X / 2, Y / 3, Z > 1 ? 1u : 0u, 0, 0};
        uint32_t ub[KLB_DATA_DIMS] = {X - 1, Y - 1, Z - 1, 0, 0};
        const size_t rx = ub[0] - lb[0] + 1, ry = ub[1] - lb[1] + 1, rz = ub[2] - lb[2] + 1;
        std::vector<uint16_t> roi(rx * ry * rz);
        check(readKLBroiInPlace(mex.c_str(), roi.data(), lb, ub, -1) == 0, "readKLBroiInPlace rc 0");
        bool same = true;
        for (size_t z = 0; z < rz; ++z)
            for (size_t y = 0; y < ry; ++y)
                same &= std::memcmp(&roi[(z * ry + y) * rx], &img[((lb[2] + z) * Y + lb[1] + y) * X + lb[0]], rx * 2) == 0;
        check(same, "readKLBroiInPlace equals the crop");
    }

    // 5. readKLBheader
    {
        uint32_t rx[KLB_DATA_DIMS], rb[KLB_DATA_DIMS];
        float32_t rps[KLB_DATA_DIMS];
        KLB_DATA_TYPE dt;
        KLB_COMPRESSION_TYPE ct;
        char rmeta[KLB_METADATA_SIZE];
        check(readKLBheader(klb.c_str(), rx, &dt, rps, rb, &ct, rmeta) == 0 && rx[0] == X && rb[0] == std::min(96u, X),
              "readKLBheader");
    }
    // 6. selection helpers on frame 0 (device buffers)
    {
        klb_imageIO io(mex);
        io.header.setHeader(xyzct, UINT16_TYPE, ps, nullptr, BZIP2, meta);
        io.header.xyzct[2] = 1;  // one frame, as writeImage's selection (klb_imageIO.cpp:2319-2327)
        io.header.Nnum = 13;
        const size_t fp = (size_t)X * Y;
        uint16_t* d_in = nullptr;
        uint16_t* d_c[8] = {nullptr};
        bool ok = hipMalloc((void**)&d_in, fp * 2) == 0 && hipMemcpy(d_in, img.data(), fp * 2, 1) == 0;
        for (int k = 0; k < 8 && ok; ++k) ok = hipMalloc((void**)&d_c[k], fp * 2) == 0;
        check(ok, "device buffers for the selection helpers");
        if (ok) {
            float raw = 0.f, scaled = 0.f, src = 0.f;
            const float r0 = io.bwt_entropy_2D(d_in, &scaled, 0);
            const float r1 = io.bwt_entropy_2D(d_in, &src, 1);
            raw = r0;
            check(r0 >= 0.f && r0 == r1 && src == raw, "bwt_entropy_2D is_src 1 reports the unscaled entropy");
            check(scaled == (float)((double)raw * 0.96), "bwt_entropy_2D is_src 0 reports (float)(e * 0.96) in double");
            std::printf("INFO bwt_entropy_2D raw %.9g scaled %.9g (float-literal product %.9g)\n", raw, scaled,
                        raw * 0.96f);
            float ent[8] = {0};
            std::atomic<uint64_t> next(0);
            check(io.predict_and_2DEntropy(d_in, d_c, ent, &next, 8) == 0, "predict_and_2DEntropy rc 0");
            float sel[8] = {0};
            int chosen = -1;
            check(lfm_hip_select(d_in, (int)X, (int)Y, 13, lfm_get_family(), sel, &chosen, nullptr, nullptr) == 0,
                  "lfm_hip_select rc 0");
            bool same = true;
            for (int k = 0; k < 8; ++k) same &= ent[k] == sel[k];
            check(same && ent[0] == scaled, "predict_and_2DEntropy entropies equal lfm_hip_select's");
            std::printf("INFO entropies");
            for (int k = 0; k < 8; ++k) std::printf(" %.9g", ent[k]);
            std::printf(" chosen %d\n", chosen);
        }
        for (int k = 0; k < 8; ++k)
            if (d_c[k]) (void)hipFree(d_c[k]);
        if (d_in) (void)hipFree(d_in);
    }
    std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED", failures);
    return failures ? 1 : 0;
}

// klb_imageHeader.cpp -- .lfm header: defaults, geometry helpers, (de)serialisation.
// Field semantics follow the reference (src/klb_imageHeader.cpp); block counts
// use the reference's float ceil (calculateNumBlocks) so Nb is identical.
#include "klb_imageHeader.h"
#include <algorithm>
#include <cmath>
#include <fstream>
#include <istream>
#include <limits>
#include <ostream>

namespace {
constexpr size_t kFixedBytes = 320;

template <class T>
void put(unsigned char*& p, const T& v)
{
    std::memcpy(p, &v, sizeof(T));
    p += sizeof(T);
}
template <class T>
void get(const unsigned char*& p, T& v)
{
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
}
} // namespace

klb_image_header::klb_image_header() : blockOffset(nullptr), Nb(0)
{
    const std::uint32_t zeros[KLB_DATA_DIMS] = {0, 0, 0, 0, 0};
    setHeader(zeros, UINT16_TYPE);
}

klb_image_header::klb_image_header(const klb_image_header& p) : blockOffset(nullptr), Nb(0)
{
    *this = p;
}

klb_image_header::~klb_image_header()
{
    delete[] blockOffset;
}

klb_image_header& klb_image_header::operator=(const klb_image_header& p)
{
    if (this == &p) return *this;
    std::memcpy(optimalBlockSizeInBytes, p.optimalBlockSizeInBytes, sizeof(optimalBlockSizeInBytes));
    setHeader(p.xyzct, p.dataType, p.pixelSize, p.blockSize, p.compressionType, p.metadata, p.headerVersion, p.Nnum);
    resizeBlockOffset(p.Nb);
    if (Nb) std::memcpy(blockOffset, p.blockOffset, Nb * sizeof(std::uint64_t));
    return *this;
}

void klb_image_header::setOptimalBlockSizeInBytes()
{
    const std::uint32_t v[KLB_DATA_DIMS] = {192, 192, 16, 1, 1};  // klb_imageHeader.h:79
    std::memcpy(optimalBlockSizeInBytes, v, sizeof(v));
}

size_t klb_image_header::calculateNumBlocks() const
{
    size_t n = 1;
    for (int d = 0; d < KLB_DATA_DIMS; ++d)
        n *= (size_t)std::ceil((float)xyzct[d] / (float)blockSize[d]);
    return n;
}

size_t klb_image_header::getBytesPerPixel() const
{
    switch (dataType) {
    case UINT8_TYPE: case INT8_TYPE: return 1;
    case UINT16_TYPE: case INT16_TYPE: return 2;
    case UINT32_TYPE: case INT32_TYPE: case FLOAT32_TYPE: return 4;
    case UINT64_TYPE: case INT64_TYPE: case FLOAT64_TYPE: return 8;
    }
    return 0;
}

std::uint32_t klb_image_header::getBlockSizeBytes() const
{
    std::uint32_t n = 1;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) n *= blockSize[d];
    return n * (std::uint32_t)getBytesPerPixel();
}

std::uint64_t klb_image_header::getImageSizePixels() const
{
    std::uint64_t n = 1;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) n *= xyzct[d];
    return n;
}

std::uint64_t klb_image_header::getImageSizeBytes() const { return getImageSizePixels() * getBytesPerPixel(); }

size_t klb_image_header::getBlockCompressedSizeBytes(size_t i) const
{
    if (i >= Nb) return 0;
    return i == 0 ? blockOffset[0] : blockOffset[i] - blockOffset[i - 1];
}

std::uint64_t klb_image_header::getBlockOffset(size_t i) const
{
    if (i >= Nb) return std::numeric_limits<std::uint64_t>::max();
    return i == 0 ? 0 : blockOffset[i - 1];
}

std::uint64_t klb_image_header::getCompressedFileSizeInBytes() const
{
    return getSizeInBytes() + (Nb ? blockOffset[Nb - 1] : 0);
}

void klb_image_header::setDefaultBlockSize()
{
    setOptimalBlockSizeInBytes();
    const std::uint32_t bpp = (std::uint32_t)std::max<size_t>(getBytesPerPixel(), 1);
    for (int d = 0; d < KLB_DATA_DIMS; ++d) blockSize[d] = std::max<std::uint32_t>(optimalBlockSizeInBytes[d] / bpp, 1);
}

void klb_image_header::resizeBlockOffset(size_t n)
{
    if (n == Nb && (blockOffset || n == 0)) return;
    delete[] blockOffset;
    blockOffset = n ? new std::uint64_t[n]() : nullptr;
    Nb = n;
}

char* klb_image_header::cloneMetadata() const
{
    char* p = new char[KLB_METADATA_SIZE];
    std::memcpy(p, metadata, KLB_METADATA_SIZE);
    return p;
}

void klb_image_header::setHeader(const std::uint32_t xyzct_[KLB_DATA_DIMS], const KLB_DATA_TYPE dataType_,
                                 const float32_t pixelSize_[KLB_DATA_DIMS], const std::uint32_t blockSize_[KLB_DATA_DIMS],
                                 const KLB_COMPRESSION_TYPE compressionType_, const char metadata_[KLB_METADATA_SIZE],
                                 const std::uint8_t headerVersion_, const std::uint8_t Nnum_)
{
    std::memcpy(xyzct, xyzct_, sizeof(xyzct));
    dataType = dataType_;
    compressionType = compressionType_;
    headerVersion = headerVersion_;
    Nnum = Nnum_;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) pixelSize[d] = pixelSize_ ? pixelSize_[d] : 1.0f;
    if (metadata_) std::memcpy(metadata, metadata_, KLB_METADATA_SIZE);
    else std::memset(metadata, 0, KLB_METADATA_SIZE);
    if (blockSize_) std::memcpy(blockSize, blockSize_, sizeof(blockSize));
    else setDefaultBlockSize();
}

size_t klb_image_header::serialize(void* out, size_t cap) const
{
    const size_t need = getSizeInBytes();
    if (!out || cap < need) return need;
    unsigned char* p = (unsigned char*)out;
    put(p, headerVersion);
    put(p, Nnum);
    for (auto v : xyzct) put(p, v);
    for (auto v : pixelSize) put(p, v);
    put(p, (std::uint8_t)dataType);
    put(p, (std::uint8_t)compressionType);
    std::memcpy(p, metadata, KLB_METADATA_SIZE);
    p += KLB_METADATA_SIZE;
    for (auto v : blockSize) put(p, v);
    if (Nb) std::memcpy(p, blockOffset, Nb * sizeof(std::uint64_t));
    return need;
}

void klb_image_header::writeHeader(FILE* fid)
{
    std::string buf(getSizeInBytes(), '\0');
    serialize(&buf[0], buf.size());
    std::fwrite(buf.data(), 1, buf.size(), fid);
}

void klb_image_header::writeHeader(std::ostream& fid)
{
    // the reference's ostream variant omits headerVersion, Nnum and metadata
    // (klb_imageHeader.cpp:153-161); kept for API compatibility
    fid.write((const char*)xyzct, sizeof(xyzct));
    fid.write((const char*)pixelSize, sizeof(pixelSize));
    const std::uint8_t dt = (std::uint8_t)dataType, ct = (std::uint8_t)compressionType;
    fid.write((const char*)&dt, 1);
    fid.write((const char*)&ct, 1);
    fid.write((const char*)blockSize, sizeof(blockSize));
    if (Nb) fid.write((const char*)blockOffset, Nb * sizeof(std::uint64_t));
}

int klb_image_header::parseHeader(const void* buf, size_t len)
{
    if (len < kFixedBytes) return 2;
    const unsigned char* p = (const unsigned char*)buf;
    std::uint8_t dt = 0, ct = 0;
    get(p, headerVersion);
    get(p, Nnum);
    for (auto& v : xyzct) get(p, v);
    for (auto& v : pixelSize) get(p, v);
    get(p, dt);
    get(p, ct);
    dataType = (KLB_DATA_TYPE)dt;
    compressionType = (KLB_COMPRESSION_TYPE)ct;
    std::memcpy(metadata, p, KLB_METADATA_SIZE);
    p += KLB_METADATA_SIZE;
    for (auto& v : blockSize) get(p, v);
    for (int d = 0; d < KLB_DATA_DIMS; ++d)
        if (blockSize[d] == 0) return 2;
    resizeBlockOffset(calculateNumBlocks());
    if (len < kFixedBytes + Nb * sizeof(std::uint64_t)) return 2;
    if (Nb) std::memcpy(blockOffset, p, Nb * sizeof(std::uint64_t));
    return 0;
}

void klb_image_header::readHeader(std::istream& fid)
{
    std::string fixed(kFixedBytes, '\0');
    fid.read(&fixed[0], kFixedBytes);
    // parse the fixed part first to learn Nb, then the offsets
    std::uint32_t bs[KLB_DATA_DIMS], xs[KLB_DATA_DIMS];
    std::memcpy(xs, fixed.data() + 2, sizeof(xs));
    std::memcpy(bs, fixed.data() + 300, sizeof(bs));
    size_t nb = 1;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) nb *= bs[d] ? (size_t)std::ceil((float)xs[d] / (float)bs[d]) : 0;
    std::string all = fixed;
    all.resize(kFixedBytes + nb * sizeof(std::uint64_t));
    if (nb) fid.read(&all[kFixedBytes], nb * sizeof(std::uint64_t));
    parseHeader(all.data(), all.size());
}

int klb_image_header::readHeader(const char* filename)
{
    std::ifstream fid(filename, std::ios::binary | std::ios::in);
    if (!fid.is_open()) {
        std::printf("ERROR: klb_image_header::readHeader : file %s could not be opened to read header\n", filename);
        return 2;
    }
    std::string fixed(kFixedBytes, '\0');
    fid.read(&fixed[0], kFixedBytes);
    if ((size_t)fid.gcount() != kFixedBytes) return 2;
    std::uint32_t bs[KLB_DATA_DIMS], xs[KLB_DATA_DIMS];
    std::memcpy(xs, fixed.data() + 2, sizeof(xs));
    std::memcpy(bs, fixed.data() + 300, sizeof(bs));
    size_t nb = 1;
    for (int d = 0; d < KLB_DATA_DIMS; ++d) {
        if (!bs[d]) return 2;
        nb *= (size_t)std::ceil((float)xs[d] / (float)bs[d]);
    }
    std::string all = fixed;
    all.resize(kFixedBytes + nb * sizeof(std::uint64_t));
    if (nb) {
        fid.read(&all[kFixedBytes], nb * sizeof(std::uint64_t));
        if ((size_t)fid.gcount() != nb * sizeof(std::uint64_t)) return 2;
    }
    return parseHeader(all.data(), all.size());
}

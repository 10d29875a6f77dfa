/*
 * klb_imageHeader.h -- in-memory form of the .lfm header.
 *
 * Public members and methods follow the reference class
 * (src/klb_imageHeader.h:35-96) because the MEX sources read and write them
 * directly (matlabWrapper/writeLFMstack.cpp:56-448).  On-disk layout
 * (little endian, 320 fixed bytes + 8 * Nb):
 *   u8 headerVersion | u8 Nnum | u32 xyzct[5] | f32 pixelSize[5] | u8 dataType |
 *   u8 compressionType | char metadata[256] | u32 blockSize[5] | u64 blockOffset[Nb]
 * blockOffset[i] is the END offset of block i, counted from the end of the header.
 */
#ifndef LFM_KLB_IMAGE_HEADER_H
#define LFM_KLB_IMAGE_HEADER_H

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iosfwd>
#include "common.h"

class __attribute__((visibility("default"))) klb_image_header
{
public:
    std::uint8_t headerVersion;                 // bit 7: video; bits 0-6: predictor request
    std::uint8_t Nnum;                          // microlens pitch in pixels
    std::uint32_t xyzct[KLB_DATA_DIMS];
    float32_t pixelSize[KLB_DATA_DIMS];
    KLB_DATA_TYPE dataType;
    KLB_COMPRESSION_TYPE compressionType;
    char metadata[KLB_METADATA_SIZE];
    std::uint32_t blockSize[KLB_DATA_DIMS];
    std::uint64_t* blockOffset;                 // Nb entries
    size_t Nb;

    klb_image_header();
    klb_image_header(const klb_image_header& p);
    ~klb_image_header();
    klb_image_header& operator=(const klb_image_header& p);

    void writeHeader(std::ostream& fid);        // reference layout of the ostream variant (no version/Nnum)
    void writeHeader(FILE* fid);                // full .lfm header
    void readHeader(std::istream& fid);
    int readHeader(const char* filename);       // 0 ok, 2 cannot open
    int parseHeader(const void* buf, size_t len);  // from memory; 0 ok, 2 truncated
    size_t serialize(void* out, size_t cap) const; // full header bytes; returns size

    size_t getNumBlocks() const { return Nb; }
    int getMetadataSizeInBytes() const { return KLB_METADATA_SIZE; }
    size_t calculateNumBlocks() const;
    size_t getSizeInBytes() const { return getSizeInBytesFixPortion() + Nb * sizeof(std::uint64_t); }
    size_t getSizeInBytesFixPortion() const { return 320; }
    size_t getBytesPerPixel() const;
    std::uint32_t getBlockSizeBytes() const;
    std::uint64_t getImageSizeBytes() const;
    std::uint64_t getImageSizePixels() const;
    size_t getBlockCompressedSizeBytes(size_t blockId) const;
    std::uint64_t getBlockOffset(size_t blockIdx) const;
    std::uint64_t getCompressedFileSizeInBytes() const;
    void setDefaultBlockSize();
    void resizeBlockOffset(size_t Nb_);
    void setOptimalBlockSizeInBytes();

    char* getMetadataPtr() { return metadata; }
    char* cloneMetadata() const;
    void setMetadata(char meta[KLB_METADATA_SIZE]) { std::memcpy(metadata, meta, KLB_METADATA_SIZE); }

    void setHeader(const std::uint32_t xyzct_[KLB_DATA_DIMS], const KLB_DATA_TYPE dataType_,
                   const float32_t pixelSize_[KLB_DATA_DIMS] = nullptr,
                   const std::uint32_t blockSize_[KLB_DATA_DIMS] = nullptr,
                   const KLB_COMPRESSION_TYPE compressionType_ = BZIP2,
                   const char metadata_[KLB_METADATA_SIZE] = nullptr,
                   const std::uint8_t headerVersion_ = KLB_DEFAULT_HEADER_VERSION, const std::uint8_t Nnum_ = 13);

private:
    std::uint32_t optimalBlockSizeInBytes[KLB_DATA_DIMS];
};

#endif

// Minimal Level-5 MAT-file writer for the acquisition dump (dump_results,
// pcps_acquisition.cc:408-508) and the tracking dump's conversion (save_matfile,
// dll_pll_veml_tracking.cc:1511-1729).  The reference writes its .mat files through
// matio (MAT_FT_MAT73, zlib-compressed); matio is not on this image, so the dump
// is written as an uncompressed Level-5 MAT-file with the same variable names,
// classes and dimensions -- MATLAB, Octave and scipy.io.loadmat read both the
// same way.  Layout (MAT-File Format, Level 5): a 128-byte header, then one
// miMATRIX element per variable: array flags (class), dimensions, name, real part,
// each sub-element padded to 8 bytes; data column-major.
#ifndef GSDR_HOST_MAT5_WRITER_H
#define GSDR_HOST_MAT5_WRITER_H

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

class Mat5Writer
{
public:
    enum Class : uint8_t
    {
        kDouble = 6,  // mxDOUBLE_CLASS
        kSingle = 7,  // mxSINGLE_CLASS
        kInt32 = 12,  // mxINT32_CLASS
        kUint32 = 13, // mxUINT32_CLASS
        kUint64 = 15  // mxUINT64_CLASS
    };

    // false when the file cannot be created
    bool open(const std::string& path);
    // a rows x cols matrix of `cls` from column-major data
    void write(const std::string& name, Class cls, uint32_t rows, uint32_t cols, const void* data);
    void write_single(const std::string& name, float v) { write(name, kSingle, 1, 1, &v); }
    void write_int32(const std::string& name, int32_t v) { write(name, kInt32, 1, 1, &v); }
    void write_uint32(const std::string& name, uint32_t v) { write(name, kUint32, 1, 1, &v); }
    void write_uint64(const std::string& name, uint64_t v) { write(name, kUint64, 1, 1, &v); }
    bool close();
    ~Mat5Writer() { close(); }

private:
    FILE* f_{nullptr};
    bool ok_{true};
};

#endif

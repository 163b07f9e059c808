#include "mat5_writer.h"

#include <cstring>

namespace
{
// data types of the sub-elements (MAT-File Format, Table 1-1)
constexpr uint32_t miINT8 = 1, miINT32 = 5, miUINT32 = 6, miSINGLE = 7, miDOUBLE = 9, miUINT64 = 13, miMATRIX = 14;

uint32_t pad8(uint32_t n) { return (n + 7u) & ~7u; }

uint32_t elem_type(Mat5Writer::Class c)
{
    switch (c)
        {
        case Mat5Writer::kSingle: return miSINGLE;
        case Mat5Writer::kInt32: return miINT32;
        case Mat5Writer::kUint32: return miUINT32;
        case Mat5Writer::kDouble: return miDOUBLE;
        default: return miUINT64;
        }
}

uint32_t elem_bytes(Mat5Writer::Class c) { return c == Mat5Writer::kUint64 || c == Mat5Writer::kDouble ? 8u : 4u; }
}  // namespace

bool Mat5Writer::open(const std::string& path)
{
    close();
    f_ = std::fopen(path.c_str(), "wb");
    ok_ = f_ != nullptr;
    if (!ok_) return false;
    // 116 bytes of text, 8 bytes of subsystem offset, version 0x0100, endian "IM"
    char hdr[128];
    std::memset(hdr, ' ', sizeof hdr);
    const char* text = "MATLAB 5.0 MAT-file, written by gnss-sdr-new_amd (GNSS-SDR dump layout)";
    std::memcpy(hdr, text, std::strlen(text));
    std::memset(hdr + 116, 0, 8);
    const uint16_t version = 0x0100;
    std::memcpy(hdr + 124, &version, 2);
    hdr[126] = 'I';
    hdr[127] = 'M';
    ok_ = std::fwrite(hdr, 1, sizeof hdr, f_) == sizeof hdr;
    return ok_;
}

void Mat5Writer::write(const std::string& name, Class cls, uint32_t rows, uint32_t cols, const void* data)
{
    if (!f_ || !ok_) return;
    const uint32_t nlen = static_cast<uint32_t>(name.size());
    const uint32_t dbytes = rows * cols * elem_bytes(cls);
    // sub-elements: flags (8 + 8), dims (8 + 8), name (8 + pad8(nlen)), data (8 + pad8(dbytes))
    const uint32_t body = 16 + 16 + 8 + pad8(nlen) + 8 + pad8(dbytes);
    std::vector<uint8_t> b;
    b.reserve(8 + body);
    auto u32 = [&b](uint32_t v) {
        uint8_t t[4];
        std::memcpy(t, &v, 4);
        b.insert(b.end(), t, t + 4);
    };
    auto pad = [&b]() {
        while (b.size() % 8) b.push_back(0);
    };
    u32(miMATRIX);
    u32(body);
    u32(miUINT32);  // array flags: class in the low byte, no complex/global/logical bits
    u32(8);
    u32(static_cast<uint32_t>(cls));
    u32(0);
    u32(miINT32);  // dimensions
    u32(8);
    u32(rows);
    u32(cols);
    u32(miINT8);  // name
    u32(nlen);
    b.insert(b.end(), name.begin(), name.end());
    pad();
    u32(elem_type(cls));  // real part
    u32(dbytes);
    const auto* d = static_cast<const uint8_t*>(data);
    b.insert(b.end(), d, d + dbytes);
    pad();
    ok_ = std::fwrite(b.data(), 1, b.size(), f_) == b.size();
}

bool Mat5Writer::close()
{
    if (!f_) return ok_;
    const bool closed = std::fclose(f_) == 0;
    f_ = nullptr;
    return ok_ && closed;
}

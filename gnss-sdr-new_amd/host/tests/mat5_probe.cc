// CPU probe of the Level-5 MAT-file writer: the acquisition dump's variable set
// with known values (tests/test_host_mirror.py reads it back with scipy.io.loadmat).
#include <cstdio>
#include <vector>

#include "mat5_writer.h"

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    Mat5Writer m;
    if (!m.open(argv[1])) return 1;
    const unsigned rows = 5, cols = 3;
    std::vector<float> g(rows * cols);
    for (unsigned c = 0; c < cols; ++c)
        for (unsigned r = 0; r < rows; ++r) g[c * rows + r] = static_cast<float>(r) + 0.25F * static_cast<float>(c);
    m.write("acq_grid", Mat5Writer::kSingle, rows, cols, g.data());
    m.write_int32("doppler_max", -5000);
    m.write_single("test_statistic", 3.5F);
    m.write_uint32("PRN", 17U);
    m.write_uint64("sample_counter", 123456789012345ULL);
    return m.close() ? 0 : 1;
}

// Host-code sanitizer driver (AddressSanitizer + UBSan, CPU only): the library's host-side
// routines — operator generator, RHS, row partition, halo plan, CSR-stream tile planning —
// on ragged and degenerate inputs.  Build and run: tools/asan_host.sh
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../vt-precondition_amd/csrc/vtk_internal.hpp"

namespace vtk {
void build_tiles(const std::vector<int32_t> &indptr, int align, std::vector<int32_t> &rows, bool &has_long,
                 bool &aligned);
}

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

int main() {
    // generator: 1D, 2D, 4D (f64/f32), full and partial row ranges
    const vtk_vlasov_params cfgs[] = {
        {1, 0, {1000, 1, 1, 1}, 6.0, 0.5, 0.05, 0.25, 4.0},
        {2, 0, {64, 32, 1, 1}, 6.0, 0.5, 0.05, 0.25, 4.0},
        {2, 0, {3, 4, 1, 1}, 6.0, 0.5, 0.05, 0.25, 4.0},
        {4, 1, {6, 5, 8, 8}, 6.0, 0.5, 0.05, 0.25, 4.0},
        {4, 0, {3, 3, 4, 2}, 6.0, 0.5, 0.05, 0.25, 4.0},
    };
    for (const auto &p : cfgs) {
        int64_t n = 0, nnz = 0;
        CHECK(vtk_vlasov_size(&p, &n, &nnz) == VTK_OK);
        for (int64_t r0 : {int64_t(0), n / 3}) {
            const int64_t r1 = r0 == 0 ? n : n - n / 5;
            std::vector<int32_t> ip(r1 - r0 + 1), ix(nnz);
            std::vector<double> d(p.fp32 ? 0 : nnz);
            std::vector<float> f(p.fp32 ? nnz : 0);
            void *data = p.fp32 ? (void *)f.data() : (void *)d.data();
            CHECK(vtk_vlasov_generate(&p, r0, r1, ip.data(), ix.data(), data) == VTK_OK);
            CHECK(ip[0] == 0 && ip.back() <= nnz);
            for (int64_t k = 0; k < ip.back(); ++k) CHECK(ix[k] >= 0 && ix[k] < n);
        }
        std::vector<double> b(n);
        CHECK(vtk_rhs_splitmix(0x5EED, 0, n, b.data()) == VTK_OK);
    }
    vtk_vlasov_params bad = cfgs[1];
    bad.dim = 3;
    int64_t n = 0, nnz = 0;
    CHECK(vtk_vlasov_size(&bad, &n, &nnz) != VTK_OK);

    // ragged CSR: empty rows, long rows, random columns
    std::mt19937 rng(7);
    for (int trial = 0; trial < 20; ++trial) {
        const int64_t nr = 1 + rng() % 3000;
        std::vector<int32_t> ip(nr + 1, 0);
        for (int64_t r = 0; r < nr; ++r) {
            int len = rng() % 9 == 0 ? 0 : 1 + rng() % 12;
            if (rng() % 200 == 0) len = 5000 + rng() % 3000;   // longer than a tile
            ip[r + 1] = ip[r] + len;
        }
        std::vector<int32_t> ix(ip[nr]);
        for (auto &c : ix) c = (int32_t)(rng() % nr);
        for (int align : {1, 2, 4, 7, 8, 64}) {
            std::vector<int32_t> rows;
            bool has_long = false, aligned = true;
            vtk::build_tiles(ip, align, rows, has_long, aligned);
            CHECK(rows.front() == 0 && rows.back() == nr);
            for (size_t t = 1; t < rows.size(); ++t) CHECK(rows[t] > rows[t - 1]);
        }
        for (int world : {1, 2, 3, 8}) {
            std::vector<int64_t> offs(world + 1);
            CHECK(vtk_partition_rows(nr, ip.data(), world, 1, offs.data()) == VTK_OK);
            CHECK(offs[0] == 0 && offs[world] == nr);
            for (int rank = 0; rank < world; ++rank) {
                const int64_t a = offs[rank], e = offs[rank + 1];
                const int64_t lnnz = ip[e] - ip[a];
                int64_t nh = 0;
                CHECK(vtk_halo_plan(nr, offs.data(), world, rank, lnnz, ix.data() + ip[a], nullptr, &nh, nullptr,
                                    nullptr) == VTK_OK);
                std::vector<int64_t> cols(nh), cnt(world);
                CHECK(vtk_halo_plan(nr, offs.data(), world, rank, lnnz, ix.data() + ip[a], nullptr, &nh,
                                    cols.data(), cnt.data()) == VTK_OK);
                for (size_t k = 1; k < cols.size(); ++k) CHECK(cols[k] > cols[k - 1]);
            }
        }
    }
    for (int s = 0; s > -9; --s) CHECK(vtk_status_string(s) != nullptr);
    if (fails) std::printf("asan_host: %d failures\n", fails);
    else std::printf("asan_host: ok\n");
    return fails ? 1 : 0;
}

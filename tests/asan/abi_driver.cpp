// Host-side exercise of the libmpo.so C ABI under AddressSanitizer (no GPU): the
// population and DenseNet planners (ragged work lists, arena layouts), every
// workspace-size query and the argument checks that return before any HIP call.
// Built and run by scripts/asan_abi.sh; tests/test_abi_asan.py drives it.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/mpo.h"

static int fails = 0;
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #c, mpo_last_error()); \
            ++fails;                                                           \
        }                                                                      \
    } while (0)

int main() {
    EXPECT(std::strlen(mpo_version()) > 0);
    std::mt19937 rng(7);
    auto U = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };

    // ---- population plans: ragged members over the test_mnist space (mpiLAPI.py)
    for (int rep = 0; rep < 6; ++rep) {
        const int n = rep == 0 ? 1 : U(2, 80);
        std::vector<MpoCnnSpec> specs(n);
        for (int i = 0; i < n; ++i) {
            specs[i] = MpoCnnSpec{U(10, 50), U(2, 10), U(2, 10), U(50, 200), 1e-3f, 0.25f, (uint32_t)i, 0};
        }
        void* h = nullptr;
        const int batch = rep % 2 ? 100 : U(1, 64);
        EXPECT(mpo_pop_create(specs.data(), n, batch, &h) == 0);
        if (!h) continue;
        MpoPopSizes sz{};
        EXPECT(mpo_pop_sizes(h, &sz) == 0);
        EXPECT(sz.n_members == n && sz.batch == batch && sz.n_params > 0 && sz.act_floats > 0);
        std::vector<int64_t> offs(64, -1);
        for (int m = 0; m < n; ++m) {
            EXPECT(mpo_pop_param_layout(h, m, offs.data()) == 0);
            EXPECT(mpo_pop_act_layout(h, m, offs.data()) == 0);
        }
        EXPECT(mpo_pop_param_layout(h, n, offs.data()) != 0);   // member out of range
        EXPECT(mpo_pop_destroy(h) == 0);
    }
    {
        MpoCnnSpec bad{5, 3, 2, 100, 1e-3f, 0.25f, 0, 0};   // F below the space
        void* h = nullptr;
        const int rc = mpo_pop_create(&bad, 1, 100, &h);
        if (rc == 0) mpo_pop_destroy(h);
        EXPECT(mpo_pop_create(nullptr, 1, 100, &h) != 0);
        EXPECT(mpo_pop_create(&bad, 0, 100, &h) != 0);
    }

    // ---- DenseNet plans (densenet.py:135-196 geometry), odd images included
    const MpoDnArch archs[] = {{32, 32, 3, 10, 10, 3, 12, 16}, {9, 11, 2, 3, 7, 2, 5, 7}, {150, 94, 5, 3, 10, 3, 12, 16},
                               {28, 28, 1, 10, 10, 3, 12, 16}, {8, 8, 3, 4, 4, 1, 4, 4}};
    for (const auto& ar : archs) {
        for (int n : {1, 7}) {
            void* h = nullptr;
            EXPECT(mpo_dn_create(&ar, n, 20, &h) == 0);
            if (!h) continue;
            MpoDnSizes sz{};
            EXPECT(mpo_dn_sizes(h, &sz) == 0);
            EXPECT(sz.n_members == n && sz.n_layers > 0 && sz.n_params > 0);
            int32_t geom[8];
            int64_t offs[6];
            for (int i = 0; i < sz.n_layers; ++i) EXPECT(mpo_dn_layer(h, i, geom, offs) == 0);
            EXPECT(mpo_dn_layer(h, sz.n_layers, geom, offs) != 0);
            EXPECT(mpo_dn_destroy(h) == 0);
        }
    }
    {
        MpoDnArch bad{32, 32, 3, 10, 11, 3, 12, 16};   // depth not 3 N + 4
        void* h = nullptr;
        EXPECT(mpo_dn_create(&bad, 1, 20, &h) != 0);
        EXPECT(std::strlen(mpo_last_error()) > 0);
    }

    // ---- workspace queries (pure host arithmetic) and early argument checks
    for (int n : {1, 5, 16, 17, 130, 200, 256, 500, 1100, 2048})
        for (int d : {1, 5, 10, 12, 16, 32}) {
            (void)mpo_gp_prepare_ws_bytes(n, d);
            (void)mpo_gp_lml_ws_bytes(n, d, 3);
        }
    EXPECT(mpo_gp_lml_ws_bytes(0, 10, 3) == 0 && mpo_gp_lml_ws_bytes(10, 40, 3) == 0);
    EXPECT(mpo_gp_lml_io_bytes(5, 3) == (3 * 7 + 3 + 3 * 7 + 2) * sizeof(double) && mpo_gp_lml_io_bytes(0, 3) == 0);
    MpoGpModel gm{};
    gm.n = 200; gm.d = 10; gm.dp = 12; gm.np16 = 208;
    EXPECT(mpo_gp_score_ws_bytes(&gm, 1000000, 5) > 0);
    EXPECT(mpo_gp_score_ws_bytes(&gm, 1000, MPO_TOPK_MAX + 1) == 0);
    EXPECT(mpo_gp_score_ws_bytes(nullptr, 10, 1) == 0);
    double dummy[4] = {0, 0, 0, 0};
    int32_t info = 0;
    EXPECT(mpo_gp_prepare(nullptr, dummy, 1, 1, dummy, 1.0, 0.1, 0.0, 1.0, &gm, dummy, 8, nullptr) != 0);
    EXPECT(mpo_gp_lml_grad(dummy, dummy, 0, 1, dummy, 1, dummy, dummy, &info, dummy, 8, nullptr) != 0);
    EXPECT(mpo_gp_lml_grad_host(dummy, dummy, 4, 1, nullptr, 1, dummy, dummy, 8, dummy, 8, nullptr) != 0);
    EXPECT(mpo_gp_lml_grad_host(dummy, dummy, 4, 1, dummy, 1, dummy, dummy, 8, dummy, 8, nullptr) != 0);  // io too small
    EXPECT(mpo_gp_acq_score(&gm, dummy, 10, 0.0, 0.01, 1.96, 1, nullptr, nullptr, nullptr, MPO_TOPK_MAX + 1,
                            nullptr, nullptr, dummy, 8, nullptr) != 0);
    EXPECT(mpo_gp_acq_grad(&gm, dummy, 0, nullptr, 0.0, 0.01, 1.96, dummy, dummy, nullptr) != 0);
    EXPECT(mpo_chol_f64(nullptr, 4, 4, &info, nullptr) != 0);
    EXPECT(mpo_trsm_f64(dummy, 2, 2, dummy, 1, 1, 2, nullptr) != 0);

    std::printf("abi_driver: %s (%d failed checks)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}

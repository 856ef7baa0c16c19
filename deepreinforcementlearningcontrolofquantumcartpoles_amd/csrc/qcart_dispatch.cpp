// qcart_dispatch.cpp — routes (family, rows-per-lane) to the per-family kernel translation units.
#include <hip/hip_runtime.h>

#include "qcart_kargs.hpp"

namespace qcart {

int launch_fam0(int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind, const uint8_t* mask,
                double a0, double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                void* stream);
int launch_fam1(int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind, const uint8_t* mask,
                double a0, double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                void* stream);
int launch_fam2(int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind, const uint8_t* mask,
                double a0, double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                void* stream);
int launch_f32(int family, int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind,
               const uint8_t* mask, double a0, double a1, double a2, const double* k_arr, const double* m_arr,
               const double* s_arr, void* stream);

namespace {
int route(int family, int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind,
          const uint8_t* mask, double a0, double a1, double a2, const double* k_arr, const double* m_arr,
          const double* s_arr, void* stream) {
    if (a.B <= 0) return 0;
    if (a.precision == 1)
        return launch_f32(family, R, kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
    if (family == 0) return launch_fam0(R, kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
    if (family == 1) return launch_fam1(R, kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
    return launch_fam2(R, kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
}
}  // namespace

bool have_kernel(int family, int R, int precision) {
    if (precision == 1) {   // fp32: Fock families (qcart_k_f32.hip)
        if (family == 1) return R == 8 || R == 16 || R == 32;
        if (family == 0) return R == 4 || R == 8 || R == 32;
        return false;
    }
    static const int r0[] = {1, 2, 4, 8}, r1[] = {1, 2, 3, 4, 8, 16}, r2[] = {1, 2, 3, 5, 9, 17};
    const int* l = family == 0 ? r0 : (family == 1 ? r1 : r2);
    const int n = family == 0 ? 4 : 6;
    for (int i = 0; i < n; i++)
        if (l[i] == R) return true;
    return false;
}

int step_waves(int family, int R, int precision) {
    KArgs a{};
    a.B = 1;
    a.precision = precision;
    return route(family, R, 4, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, nullptr);
}

int step_dual_img(int family, int R, int precision) {
    KArgs a{};
    a.B = 1;
    a.precision = precision;
    return route(family, R, 6, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, nullptr);
}

int launch_resident(int family, int R, const KArgs& a, const ResArgs& r, void* stream) {
    return route(family, R, 7, a, 0, 0.0, (void*)&r, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, stream);
}
bool have_resident(int family, int R) {
    KArgs a{};
    a.B = 1;
    return have_kernel(family, R, 0) &&
           route(family, R, 8, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, nullptr) == 1;
}

int launch_step(int family, int R, const KArgs& a, void* stream) {
    return route(family, R, 0, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, stream);
}
int launch_obs(int family, int R, const KArgs& a, void* stream) {
    return route(family, R, 1, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, stream);
}
int launch_aux(int family, int R, int what, const KArgs& a, double xth, void* out, void* stream) {
    return route(family, R, 2, a, what, xth, out, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, stream);
}
int launch_control(int family, int R, const KArgs& a, void* stream) {
    return route(family, R, 5, a, 0, 0.0, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, nullptr, stream);
}
int launch_reset(int family, int R, const KArgs& a, int kind, const uint8_t* mask, double a0, double a1, double a2,
                 const double* k_arr, const double* m_arr, const double* s_arr, void* stream) {
    return route(family, R, 3, a, 0, 0.0, nullptr, kind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
}

}  // namespace qcart

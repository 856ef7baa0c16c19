// qcart_k_iho.hip — inverted-harmonic (IHO) Fock family: instantiations of the step / observation / aux / reset kernels.
// Split per family so the three translation units compile in parallel.
#include "qcart_kernels.hpp"

namespace qcart {

int launch_fam1(int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind, const uint8_t* mask,
                 double a0, double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                 void* stream) {
    switch (R) {
        case 1: return launch_one<1, 1>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 2: return launch_one<1, 2>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 3: return launch_one<1, 3>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 4: return launch_one<1, 4>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 8: return launch_one<1, 8>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 16: return launch_one<1, 16>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        default: return -6;
    }
}

}  // namespace qcart

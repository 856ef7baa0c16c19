// qcart_k_grid.hip — quartic grid (QO / IQO) family: instantiations of the step / observation / aux / reset kernels.
// Split per family so the three translation units compile in parallel.
#include "qcart_kernels.hpp"

namespace qcart {

int launch_fam2(int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind, const uint8_t* mask,
                 double a0, double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                 void* stream) {
    switch (R) {
        case 1: return launch_one<2, 1>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 2: return launch_one<2, 2>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 3: return launch_one<2, 3>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 5: return launch_one<2, 5>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 9: return launch_one<2, 9>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        case 17: return launch_one<2, 17>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream);
        default: return -6;
    }
}

}  // namespace qcart

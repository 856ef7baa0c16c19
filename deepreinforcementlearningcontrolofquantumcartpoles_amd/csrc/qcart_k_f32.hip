// qcart_k_f32.hip — fp32 working-precision instantiations (BASELINE config C5: IHO N = 2048, fp32) of
// the Fock-family step / observation / aux / reset kernels. Same code as the fp64 kernels
// (qcart_kernels.hpp, RT = float); factor tables are rounded from the fp64 host construction.
#include "qcart_kernels.hpp"

namespace qcart {

int launch_f32(int family, int R, int kind, const KArgs& a, int what, double xth, void* out, int rkind,
               const uint8_t* mask, double a0, double a1, double a2, const double* k_arr, const double* m_arr,
               const double* s_arr, void* stream) {
#define QC_F32(F, RR) \
    return launch_one<F, RR, float>(kind, a, what, xth, out, rkind, mask, a0, a1, a2, k_arr, m_arr, s_arr, stream)
    if (family == 1) {
        switch (R) {
            case 8: QC_F32(1, 8);
            case 16: QC_F32(1, 16);
            case 32: QC_F32(1, 32);
            default: return -6;
        }
    }
    if (family == 0) {
        switch (R) {
            case 4: QC_F32(0, 4);
            case 8: QC_F32(0, 8);
            case 32: QC_F32(0, 32);
            default: return -6;
        }
    }
#undef QC_F32
    return -6;
}

}  // namespace qcart

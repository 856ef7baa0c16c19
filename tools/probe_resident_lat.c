/* probe_resident_lat.c — one step-server client's call latency without Python: `calls` step() calls of one env at
 * n_max + 1 rows (force on the action grid: the resident kernel when the server has one), µs per call as JSON.
 *   gcc -O2 tools/probe_resident_lat.c -Ldeepreinforcementlearningcontrolofquantumcartpoles_amd -lqcart_client -o tools/bin/probe_resident_lat
 *   probe_resident_lat /name calls [force] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/qcart_client.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e6 + 1e-3 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int calls = atoi(argv[2]);
    const double force = argc > 3 ? atof(argv[3]) : 0.8;
    qcc* c = NULL;
    if (qcc_open(argv[1], &c) != QCC_OK) {
        fprintf(stderr, "open: %s\n", qcc_last_error(NULL));
        return 1;
    }
    const int N = qcc_dim(c);
    double* psi = (double*)calloc((size_t)2 * N, sizeof(double));
    double q, xm;
    int32_t fail;
    double t0 = 0.0;
    for (int i = 0; i < calls + 200; ++i) {
        if (i % 80 == 0) {   /* a fresh |0> every control interval: the trajectory stays physical */
            memset(psi, 0, sizeof(double) * 2 * (size_t)N);
            psi[0] = 1.0;
        }
        if (i == 200) t0 = now_us();
        if (qcc_step(c, psi, 1, 1.0 / 1440, force, 6.283185307179586, &q, &xm, &fail) != QCC_OK) {
            fprintf(stderr, "step: %s\n", qcc_last_error(c));
            return 1;
        }
    }
    printf("{\"N\": %d, \"force\": %g, \"us_per_call\": %.2f}\n", N, force, (now_us() - t0) / calls);
    qcc_close(c);
    return 0;
}

/* A BEAM scheduler's bind loop without an interpreter lock: `iters` calls of
 * laspj_var_etf_bind (lasp_core:bind/3, lasp_core.erl:291-312) on one variable, so that
 * threads calling it at once reach the library concurrently (bench.py's scheduler legs;
 * Python threads would serialise on the GIL between calls).  Built against
 * include/laspj.h and liblaspj.so alone. */
#include <stdint.h>

#include "../../include/laspj.h"

int bind_loop(laspj_var* var, const uint8_t* value, uint64_t n, int iters, int32_t* status,
              int32_t* verdict) {
    for (int i = 0; i < iters; ++i) {
        int s = laspj_var_etf_bind(var, value, n, status, verdict);
        if (s) return s;
        if (*verdict != LASPJ_NIF_OK) return 100;
    }
    return LASPJ_OK;
}

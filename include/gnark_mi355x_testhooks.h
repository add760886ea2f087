/* Test-only entry points: element-wise device primitives of the field / curve
 * layer, used by the parity tests (tests/test_field_gpu.py) to pin each
 * arithmetic primitive against the oracle.  Built into
 * libgnark_mi355x_testhooks.so (csrc/testhooks.hip), which links against
 * libgnark_mi355x.so; the product library does not contain them.  Not on the
 * proving path, and nothing in the reference's FFI corresponds to them. */
#ifndef GNARK_MI355X_TESTHOOKS_H
#define GNARK_MI355X_TESTHOOKS_H

#include "gnark_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kind: 0 = Fr, 1 = Fp, 2 = Fp2; op: 0 mul, 1 add, 2 sub, 3 neg, 4 inv, 5 sqr.
 * Point op (affine in/out): 0 mixed add, 1 double, 2 XYZZ add, 3 [1000003]P. */
int gm_test_field_op(gm_ctx* ctx, int curve, int kind, int op, const void* a_dev,
                     const void* b_dev, void* out_dev, size_t n);
int gm_test_point_op(gm_ctx* ctx, int curve, int g2, int op, const void* a_dev,
                     const void* b_dev, void* out_dev, size_t n);

/* Replays the level shape of the reference benchmark circuit (a chain of
 * squarings: level j finishes constraint j and solves wire nb_inputs + j)
 * through gm_g16_stage_put_indexed: mode 0 one put per level and vector, mode 1
 * the Go level hook's gathering (a put every flush_at ids); abc = 0 stages the
 * wires only.  Reports the host time per level. */
int gm_test_stage_replay_chain(gm_g16_stage* st, const void* wires, size_t nb_inputs, const void* a,
                               const void* b, const void* c, size_t nb_constraints, int mode, int abc,
                               size_t flush_at, double* ns_per_level);

#ifdef __cplusplus
}
#endif

#endif

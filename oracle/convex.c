/* convex.c — convex-hull (mesh) narrowphase.  TEST INFRASTRUCTURE ONLY.
 * Stage 1: not yet implemented — mesh pairs produce no contact (documented gap). */
#include "physics.h"
int orc_convex_collide(const pnp_model_desc* m, const orc_data* d, int g1, int g2, double margin,
                       orc_contact* out, int cap) {
  (void)m; (void)d; (void)g1; (void)g2; (void)margin; (void)out; (void)cap;
  return 0;
}

// Photon-map pre-pass entry (myScene.initRender, myScene.java:1096-1099).
#include "rt_internal.h"

extern "C" int rt_photons_build(rt_scene* s, uint64_t seed) {
  (void)seed;
  if (!s) return rt::set_error(RT_E_INVALID, "null scene");
  if (s->hs.photonMode == 0) return RT_OK;
  return rt::set_error(RT_E_INVALID, "photon maps: GPU photon pre-pass not built yet");
}

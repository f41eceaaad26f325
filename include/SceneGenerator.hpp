/* SceneGenerator.hpp -- the reference's SceneGenerator (SceneGenerator.cpp:10-56) as a library.
 * The `SceneGenerator` executable built from this repo prints the same stdout byte for byte. */
#ifndef VCRT_SCENE_GENERATOR_HPP
#define VCRT_SCENE_GENERATOR_HPP

#include <string>
#include <vector>

#include "vcrt.h"

namespace vcrt {
std::vector<vcrt_sphere> generate_random_spheres(int lo, int hi, int max_accept);
std::string scene_generator_text();
int builtin_scene(int scene_id, std::vector<vcrt_sphere>& out);
}  // namespace vcrt

#endif

// SceneGenerator executable: prints the same stdout as the reference's SceneGenerator.cpp
// (SceneGenerator.cpp:23-56), produced by the library in scene.cpp.
#include <cstdio>
#include <string>

#include "scene.hpp"

int main(void) {
    const std::string text = vcrt::scene_generator_text();
    std::fwrite(text.data(), 1, text.size(), stdout);
    return 0;
}

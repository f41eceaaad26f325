// scene.cpp -- SceneGenerator as a library (SceneGenerator.cpp:10-56) plus the built-in scenes.
//
// The reference's SceneGenerator is a standalone program whose stdout (GLSL initializers) was
// pasted into globals.glsl:31-511. Here the same generator fills vcrt_sphere[] directly and can
// still print the identical text. It uses the same libstdc++ engine and distribution as the
// reference (std::mt19937, default seed 5489, std::uniform_real_distribution<double>), with the
// argument evaluation order GCC used for the reference build made explicit: in
//   point3 center(a + 0.9*rd(), 0.2, b + 0.9*rd());   the z draw happens before the x draw,
//   printf(fmt, rd(), rd(), rd(), rd());               param is drawn first, then b, g, r.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "scene.hpp"

namespace vcrt {

namespace {

struct Generator {
    std::mt19937 engine;  // default seed 5489 (SceneGenerator.cpp:19)
    std::uniform_real_distribution<double> dist{0.0, 1.0};
    double next() { return dist(engine); }
};

struct Candidate {
    float cx, cy, cz;
    int kind;  // VCRT_TEXTURE_*
    double r, g, b, param;
};

// SceneGenerator.cpp:26-46 for one grid cell; false when the cell is skipped.
bool generate_cell(Generator& gen, int a, int b, Candidate& c) {
    const double choose_mat = gen.next();
    const double z_draw = gen.next();
    const double x_draw = gen.next();
    c.cx = static_cast<float>(a + 0.9 * x_draw);
    c.cy = static_cast<float>(0.2);
    c.cz = static_cast<float>(b + 0.9 * z_draw);
    // (center - point3(4, 0.2, 0)).length() < 0.9, with length() the SQUARED length (line 14)
    const float dx = c.cx - 4.0f, dy = c.cy - static_cast<float>(0.2), dz = c.cz - 0.0f;
    const float len2 = dx * dx + dy * dy + dz * dz;
    if (static_cast<double>(len2) < 0.9) return false;
    if (choose_mat < 0.95) {
        c.kind = choose_mat < 0.8 ? VCRT_TEXTURE_LAMBERTIAN : VCRT_TEXTURE_METAL;
        c.param = gen.next();
        c.b = gen.next();
        c.g = gen.next();
        c.r = gen.next();
    } else {
        c.kind = VCRT_TEXTURE_GLASS;
        c.r = c.g = c.b = 1.0;
        c.param = 1.5;
    }
    return true;
}

// A "%.2f" field as the GLSL compiler reads it back: a decimal literal rounded to fp32.
float as_printed(double v) {
    char tmp[64];
    std::snprintf(tmp, sizeof(tmp), "%.2f", v);
    return std::strtof(tmp, nullptr);
}

vcrt_sphere make_sphere(float cx, float cy, float cz, float r, float cr, float cg, float cb,
                        int kind, float param) {
    vcrt_sphere s;
    s.center[0] = cx;
    s.center[1] = cy;
    s.center[2] = cz;
    s.radius = r;
    s.colour[0] = cr;
    s.colour[1] = cg;
    s.colour[2] = cb;
    s.texture[0] = static_cast<float>(kind);
    s.texture[1] = param;
    s.texture[2] = 0.0f;
    return s;
}

// globals.glsl:513-517
vcrt_sphere big_glass() { return make_sphere(0, 1, 0, 1.0f, 1.0f, 1.0f, 1.0f, 3, 1.5f); }
vcrt_sphere big_lambertian() {
    return make_sphere(-4, 1, 0, 1.0f, 0.4f, 0.2f, 0.1f, 1, 1.0f);
}
vcrt_sphere big_metal() { return make_sphere(4, 1, 0, 1.0f, 0.7f, 0.6f, 0.5f, 2, 1.0f); }
vcrt_sphere ground() { return make_sphere(0, -1000, 0, 1000, 0.5f, 0.5f, 0.5f, 1, 1.0f); }

}  // namespace

std::vector<vcrt_sphere> generate_random_spheres(int lo, int hi, int max_accept) {
    Generator gen;
    std::vector<vcrt_sphere> out;
    for (int a = lo; a < hi; a++) {
        for (int b = lo; b < hi; b++) {
            if (max_accept > 0 && static_cast<int>(out.size()) >= max_accept) return out;
            Candidate c;
            if (!generate_cell(gen, a, b, c)) continue;
            if (c.kind == VCRT_TEXTURE_GLASS) {
                out.push_back(make_sphere(as_printed(c.cx), as_printed(c.cy), as_printed(c.cz),
                                          0.2f, 1.0f, 1.0f, 1.0f, c.kind, 1.5f));
            } else {
                out.push_back(make_sphere(as_printed(c.cx), as_printed(c.cy), as_printed(c.cz),
                                          0.2f, as_printed(c.r), as_printed(c.g),
                                          as_printed(c.b), c.kind, as_printed(c.param)));
            }
        }
    }
    return out;
}

std::string scene_generator_text() {
    Generator gen;
    std::string text;
    char line[256];
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            Candidate c;
            if (!generate_cell(gen, a, b, c)) continue;
            std::snprintf(line, sizeof(line), "sphere(vec3(%.2f,%.2f,%.2f), 0.2, ",
                          static_cast<double>(c.cx), static_cast<double>(c.cy),
                          static_cast<double>(c.cz));
            text += line;
            if (c.kind == VCRT_TEXTURE_LAMBERTIAN) {
                std::snprintf(line, sizeof(line),
                              "vec3(%.2f,%.2f,%.2f), vec3(TEXTURE_LAMBERTIAN,%.2f,0.0)),\n", c.r,
                              c.g, c.b, c.param);
            } else if (c.kind == VCRT_TEXTURE_METAL) {
                std::snprintf(line, sizeof(line),
                              "vec3(%.2f,%.2f,%.2f), vec3(TEXTURE_METAL,%.2f,0.0)),\n", c.r, c.g,
                              c.b, c.param);
            } else {
                std::snprintf(line, sizeof(line),
                              "vec3(1.0,1.0,1.0), vec3(TEXTURE_GLASS,1.5,0.0)),\n");
            }
            text += line;
        }
    }
    text += "\n";
    text += "sphere(vec3(0, 1, 0),1.0, vec3(1.0,1.0,1.0), vec3(TEXTURE_GLASS,1.5,0.0)),\n";
    text += "sphere(vec3(-4, 1, 0),1.0, vec3(0.4, 0.2, 0.1), vec3(TEXTURE_LAMBERTIAN,1.0,0.0)),\n";
    text += "sphere(vec3(4, 1, 0),1.0, vec3(0.7, 0.6, 0.5), vec3(TEXTURE_METAL,1.0,0.0)),\n";
    return text;
}

int builtin_scene(int scene_id, std::vector<vcrt_sphere>& out) {
    out.clear();
    switch (scene_id) {
        case VCRT_SCENE_FINAL:
            out = generate_random_spheres(-11, 11, 0);
            break;
        case VCRT_SCENE_THREE:
            break;
        case VCRT_SCENE_RED:
            out.push_back(make_sphere(0, 1, 0, 1.0f, 1.0f, 0.0f, 0.0f, 1, 1.0f));
            out.push_back(ground());
            return VCRT_SUCCESS;
        case VCRT_SCENE_STRESS4096:
            out = generate_random_spheres(-33, 33, 4096);
            break;
        default:
            return VCRT_ERROR_FEATURE_NOT_PRESENT;
    }
    out.push_back(big_glass());
    out.push_back(big_lambertian());
    out.push_back(big_metal());
    out.push_back(ground());
    return VCRT_SUCCESS;
}

}  // namespace vcrt

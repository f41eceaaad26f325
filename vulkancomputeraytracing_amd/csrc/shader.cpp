// shader.cpp -- CreateShaderStageFromFile for gfx950 code objects (reference: Shader.cpp:34-95).
//
// Reference behaviour kept: stat + fopen + read the whole file, error
// VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT when it cannot be read, otherwise the module-creation
// result passes through. The embedded-blob mode (LOAD_SHADER_FROM_MEMORY, Shader.cpp:13-23)
// is selected with filename == nullptr and uses the code object linked into libvcrt.so.
#include <sys/stat.h>

#include <cstdio>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "Shader.hpp"
#include "hip_status.hpp"

extern "C" const unsigned char vcrt_embedded_code_object[];
extern "C" const unsigned char vcrt_embedded_code_object_end[];

VkResult CreateShaderStageFromFile(IN const char* filename, IN VkShaderStageFlagBits stage,
                                   OUT VkPipelineShaderStageCreateInfo* info) {
    if (!info) return VK_ERROR_INITIALIZATION_FAILED;
    hipModule_t module = nullptr;
    hipError_t err;
    if (filename == nullptr) {
        err = hipModuleLoadData(&module, vcrt_embedded_code_object);
    } else {
        struct stat file_info;
        if (stat(filename, &file_info) != 0 || file_info.st_size <= 0)
            return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
        FILE* file = std::fopen(filename, "rb");
        if (!file) return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
        std::vector<unsigned char> data(static_cast<size_t>(file_info.st_size));
        const size_t got = std::fread(data.data(), 1, data.size(), file);
        std::fclose(file);
        if (got != data.size()) return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
        err = hipModuleLoadData(&module, data.data());
    }
    if (err == hipErrorInvalidImage || err == hipErrorNoBinaryForGpu ||
        err == hipErrorInvalidKernelFile || err == hipErrorSharedObjectInitFailed)
        return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
    if (err != hipSuccess) return vcrt::to_vk(err);
    info->sType = 18;  // VK_STRUCTURE_TYPE_PIPELINE_SHADER_STAGE_CREATE_INFO
    info->stage = stage;
    info->module = module;
    // The code object holds every tracer variant; which one is the entry point depends on the
    // scene and the desc (capi.cpp select_kernel), so the renderer names it: after the scene is
    // set (vcrt_set_scene, vcrt_shader_load) and at every draw. Unnamed until then.
    info->pName = nullptr;
    return VK_SUCCESS;
}

void DestroyShaderStage(IN VkPipelineShaderStageCreateInfo* info) {
    if (info && info->module) {
        (void)hipModuleUnload(static_cast<hipModule_t>(info->module));
        info->module = nullptr;
    }
}

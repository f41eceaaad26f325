/* Shader.hpp -- kernel code-object loading, the analogue of the reference's
 * CreateShaderStageFromFile (include/Shader.hpp:14-15, Shader.cpp:34-95).
 *
 * The reference reads a SPIR-V file relative to the working directory (or an embedded blob
 * under LOAD_SHADER_FROM_MEMORY) and wraps it into a pipeline stage with entry point "main".
 * Here the file is a gfx950 code object (.hsaco) and the "stage" is the HIP module holding the
 * tracer kernels. Same error convention: VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT when the file
 * cannot be read (Shader.cpp:61,67) or is not loadable; other failures pass through. */
#ifndef VCRT_SHADER_HPP
#define VCRT_SHADER_HPP

#include "Common.hpp"

typedef enum VkShaderStageFlagBits {
    VK_SHADER_STAGE_COMPUTE_BIT = 0x00000020
} VkShaderStageFlagBits;

typedef struct VkPipelineShaderStageCreateInfo {
    int32_t sType;
    VkShaderStageFlagBits stage;
    void* module;      /* hipModule_t */
    const char* pName; /* the tracer entry point: named by the renderer for its scene and desc
                          (capi.cpp select_kernel); NULL out of CreateShaderStageFromFile */
} VkPipelineShaderStageCreateInfo;

// Load & bind. filename == nullptr selects the code object embedded in libvcrt.so.
VkResult CreateShaderStageFromFile(IN const char* filename, IN VkShaderStageFlagBits stage,
                                   OUT VkPipelineShaderStageCreateInfo* shaderStageCreateInfo);

// Releases a module returned by CreateShaderStageFromFile.
void DestroyShaderStage(IN VkPipelineShaderStageCreateInfo* shaderStageCreateInfo);

#endif

// hip_status.hpp -- hipError_t -> VkResult-compatible codes (vcrt.h), never throws.
#pragma once

#include <hip/hip_runtime_api.h>

#include "Common.hpp"

namespace vcrt {

inline VkResult to_vk(hipError_t e) {
    switch (e) {
        case hipSuccess: return VK_SUCCESS;
        case hipErrorOutOfMemory: return VK_ERROR_OUT_OF_DEVICE_MEMORY;
        case hipErrorInvalidImage:
        case hipErrorNoBinaryForGpu:
        case hipErrorInvalidKernelFile: return VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT;
        case hipErrorNoDevice:
        case hipErrorInvalidDevice:
        case hipErrorNotInitialized:
        case hipErrorInsufficientDriver: return VK_ERROR_INITIALIZATION_FAILED;
        case hipErrorLaunchFailure:
        case hipErrorIllegalAddress:
        case hipErrorLaunchTimeOut:
        case hipErrorECCNotCorrectable: return VK_ERROR_DEVICE_LOST;
        default: return VK_ERROR_UNKNOWN;
    }
}

}  // namespace vcrt

/* Common.hpp -- shared definitions of the C++ host API (mirrors include/Common.hpp of the
 * reference: IN/OUT markers, default window size, VkResult). No Vulkan headers exist here, so
 * VkResult is an int32_t carrying the same registry values (see vcrt.h). */
#ifndef VCRT_COMMON_HPP
#define VCRT_COMMON_HPP

#include <cstdint>

#include "vcrt.h"

#define IN
#define OUT

typedef int32_t VkResult;

#ifndef VK_SUCCESS
#define VK_SUCCESS VCRT_SUCCESS
#define VK_ERROR_OUT_OF_HOST_MEMORY VCRT_ERROR_OUT_OF_HOST_MEMORY
#define VK_ERROR_OUT_OF_DEVICE_MEMORY VCRT_ERROR_OUT_OF_DEVICE_MEMORY
#define VK_ERROR_INITIALIZATION_FAILED VCRT_ERROR_INITIALIZATION_FAILED
#define VK_ERROR_DEVICE_LOST VCRT_ERROR_DEVICE_LOST
#define VK_ERROR_FEATURE_NOT_PRESENT VCRT_ERROR_FEATURE_NOT_PRESENT
#define VK_ERROR_FORMAT_NOT_SUPPORTED VCRT_ERROR_FORMAT_NOT_SUPPORTED
#define VK_ERROR_UNKNOWN VCRT_ERROR_UNKNOWN
#define VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT VCRT_ERROR_INCOMPATIBLE_SHADER_BINARY
#endif

/* include/Common.hpp:23-25 of the reference */
constexpr auto WINDOW_WIDTH = 1280;
constexpr auto WINDOW_HEIGHT = 720;
constexpr auto RENDER_ITERATION = 100;

#endif

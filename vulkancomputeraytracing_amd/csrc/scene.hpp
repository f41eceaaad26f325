// scene.hpp -- internal include of the SceneGenerator library API.
#pragma once
#include "SceneGenerator.hpp"

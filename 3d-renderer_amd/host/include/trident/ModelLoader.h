// ModelLoader.h — geometry ingestion without Assimp.
//
// The reference imports models with Assimp 5.3.1 (Trident/src/Loader/ModelLoader.cpp:331, flags
// :26-37) and textures with stb_image (TextureLoader.cpp:290-304). Neither library is vendored in the
// reference snapshot, so this restates the parts of their behaviour that reach the renderer:
//   - ModelData / MeshInstance with the reference's field names (ModelLoader.h:21-40);
//   - Wavefront OBJ + MTL and glTF 2.0 (.gltf with external or data-URI buffers, .glb);
//   - aiProcess_Triangulate (polygon fans), aiProcess_JoinIdenticalVertices (exact attribute match),
//     aiProcess_GenSmoothNormals (normalised face normals summed per position when the file has none),
//     aiProcess_CalcTangentSpace (per-triangle UV tangents summed per vertex; the shaders never read
//     them, Default.frag:126-130), missing vertex colours = white (ModelLoader.cpp:436-443);
//   - material mapping: base colour (glTF baseColorFactor, MTL Kd + d), metallic / roughness (glTF
//     factors, MTL Pm / Pr; defaults 1 / 1 as ModelLoader.cpp:375-378), base-colour texture path;
//   - glTF node hierarchy baked into MeshInstance matrices (ModelLoader.cpp:505-540).
// Not restated: aiProcess_ImproveCacheLocality / OptimizeMeshes (they only reorder triangles or merge
// meshes; the rendered image differs at most at exact depth ties), skeletons and animation clips.
// Images: binary PPM (P6) and PAM (P7, RGB / RGBA) decode to forced RGBA8 with stb's vertical flip
// (stbi_set_flip_vertically_on_load, TextureLoader.cpp:290-304); PNG / JPEG need stb and fail to load
// (the renderer then uses the default slot, as the reference does after a failed load).
#pragma once

#include <limits>
#include <string>
#include <vector>

#include "Scene.h"

namespace Trident {
namespace Loader {

struct MeshInstance {
    size_t m_MeshIndex = std::numeric_limits<size_t>::max();
    glm::mat4 m_ModelMatrix{1.0f};
    std::string m_NodeName;
};

struct ModelData {
    std::vector<Geometry::Mesh> m_Meshes;
    std::vector<Geometry::Material> m_Materials;
    std::vector<std::string> m_Textures;  // normalised paths referenced by materials
    std::vector<MeshInstance> m_MeshInstances;
};

class ModelLoader {
public:
    // Empty ModelData (and a logged error) when the file is missing, unsupported or malformed.
    static ModelData Load(const std::string& filePath);
};

class TextureLoader {
public:
    // RGBA8, rows flipped bottom-up like stb with flip-on-load; Width = 0 on failure.
    static TextureData Load(const std::string& filePath);
};

// ApplicationLayer's DecomposeMatrixToTransform (ApplicationLayer.cpp:838-861): glm::decompose, then
// degrees(eulerAngles(normalize(q))). Returns false (and the default transform) when it fails.
bool DecomposeMatrixToTransform(const glm::mat4& modelMatrix, Transform& out);

}  // namespace Loader
}  // namespace Trident

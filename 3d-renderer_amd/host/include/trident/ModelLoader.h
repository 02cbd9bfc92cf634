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
// Images: PNG (ImageDecoder.h: stb_image's PNG semantics on zlib) and binary PPM (P6) / PAM (P7, RGB /
// RGBA) decode to forced RGBA8 with stb's vertical flip for 2D textures (stbi_set_flip_vertically_on_load,
// TextureLoader.cpp:290-304) and without it for cube faces (:773); JPEG / TGA / BMP / HDR need stb and
// fail to load (the renderer then uses the default slot, as the reference does after a failed load).
#pragma once

#include <array>
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

// SkyboxTextureLoader (TextureLoader.h / TextureLoader.cpp:334-830), LDR faces: every face decoded to
// RGBA8 without the vertical flip, all faces of one size, stored +X,-X,+Y,-Y,+Z,-Z. An invalid (empty)
// result and a logged error when a face is missing, fails to decode or differs in size. EXR and KTX
// need tinyexr / a KTX parser that are not restated: such inputs load as invalid.
class SkyboxTextureLoader {
public:
    static CubemapTextureData LoadFromFaces(const std::array<std::string, 6>& facePaths);
    // TryMatchFaceIndex (:140-160) per file of the directory (sorted order): the first face whose
    // token (posx/px, negx/nx, ...) the lower-case stem contains; the first candidate per face wins.
    static CubemapTextureData LoadFromDirectory(const std::string& directoryPath);
};

// Renderer::CreateSkyboxCubemap's discovery (Renderer.cpp:3830-3927) under `assetsDir` (the reference
// uses "Assets", relative to the working directory): Skyboxes/DefaultSkybox.ktx, else the
// Skyboxes/Default directory, else loose PNG faces in Skyboxes/ matched by the px/nx/... tokens (a
// file may fill every still-missing face whose token its stem contains), else invalid. `source`
// names what was used ("DefaultSkybox.ktx", "Default directory", "PNG fallback" or "").
CubemapTextureData DiscoverDefaultSkybox(const std::string& assetsDir, std::string& source);

// ApplicationLayer's DecomposeMatrixToTransform (ApplicationLayer.cpp:838-861): glm::decompose, then
// degrees(eulerAngles(normalize(q))). Returns false (and the default transform) when it fails.
bool DecomposeMatrixToTransform(const glm::mat4& modelMatrix, Transform& out);

}  // namespace Loader
}  // namespace Trident

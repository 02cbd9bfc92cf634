// ModelLoader.cpp — OBJ/MTL and glTF 2.0 ingestion + PPM/PAM textures (see ModelLoader.h for the
// Assimp / stb behaviour restated here and what is not).
#include "trident/ModelLoader.h"
#include "trident/ImageDecoder.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <unordered_map>

namespace Trident {
namespace Loader {

namespace {

namespace fs = std::filesystem;

void LogError(const char* what, const std::string& detail) {
    std::fprintf(stderr, "[Trident][ModelLoader] %s: %s\n", what, detail.c_str());
}

// Utilities::FileManagement::NormalizePath (Core/Utilities.cpp:390-394)
std::string NormalizePath(const std::string& path) { return fs::path(path).lexically_normal().generic_string(); }

std::string Lower(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return s;
}

bool ReadFile(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// ResolveTextureIndex (ModelLoader.cpp:219-261): relative paths resolve against the model's
// directory, normalised, de-duplicated; '*N' embedded references are unsupported.
int ResolveTextureIndex(const std::string& raw, const fs::path& modelDirectory, ModelData& data,
                        std::unordered_map<std::string, int>& lookup) {
    if (raw.empty()) return -1;
    fs::path p{raw};
    if (raw.front() == '*') {
        LogError("embedded textures are not supported", raw);
        return -1;
    }
    if (!p.is_absolute()) p = modelDirectory / p;
    const std::string n = NormalizePath(p.string());
    if (n.empty()) return -1;
    auto it = lookup.find(n);
    if (it != lookup.end()) return it->second;
    const int index = (int)data.m_Textures.size();
    data.m_Textures.push_back(n);
    lookup.emplace(n, index);
    return index;
}

// ---- post-processing shared by both importers --------------------------------------------------
struct Corner {  // one triangle corner before aiProcess_JoinIdenticalVertices
    glm::vec3 p, n, c;
    glm::vec2 uv;
    bool hasNormal;
};

// aiProcess_GenSmoothNormals (only when the mesh has no normals): each face's normalised normal is
// added to every corner that shares the corner's position; the sum is normalised.
void GenSmoothNormals(std::vector<Corner>& corners) {
    struct Key {
        float x, y, z;
        bool operator<(const Key& o) const {
            return std::memcmp(this, &o, sizeof(Key)) < 0;
        }
    };
    std::map<Key, glm::vec3> sum;
    std::vector<glm::vec3> faceN(corners.size() / 3);
    for (size_t t = 0; t + 2 < corners.size(); t += 3) {
        const glm::vec3 e1 = corners[t + 1].p - corners[t].p, e2 = corners[t + 2].p - corners[t].p;
        glm::vec3 n = glm::cross(e1, e2);
        const float len = glm::length(n);
        n = len > 0.0f ? n * (1.0f / len) : glm::vec3(0.0f);
        faceN[t / 3] = n;
        for (int k = 0; k < 3; ++k) {
            const glm::vec3& p = corners[t + k].p;
            glm::vec3& s = sum[Key{p.x, p.y, p.z}];
            s = s + n;
        }
    }
    for (Corner& c : corners) {
        glm::vec3 s = sum[Key{c.p.x, c.p.y, c.p.z}];
        const float len = glm::length(s);
        c.n = len > 0.0f ? s * (1.0f / len) : glm::vec3(0.0f);
        c.hasNormal = true;
    }
}

// Triangle corners -> indexed Geometry::Mesh with exact-match vertex welding
// (aiProcess_JoinIdenticalVertices), then per-vertex tangent frames (aiProcess_CalcTangentSpace).
Geometry::Mesh BuildMesh(std::vector<Corner>& corners, bool hasNormals, int materialIndex) {
    if (!hasNormals) GenSmoothNormals(corners);
    Geometry::Mesh mesh;
    mesh.MaterialIndex = materialIndex;
    std::map<std::string, uint32_t> weld;
    mesh.Indices.reserve(corners.size());
    for (const Corner& c : corners) {
        Vertex v{};
        v.Position = c.p;
        v.Normal = c.n;
        v.Color = c.c;
        v.TexCoord = c.uv;
        std::string key(reinterpret_cast<const char*>(&v), offsetof(Vertex, Tangent));
        key.append(reinterpret_cast<const char*>(&v.Color), sizeof(glm::vec3) + sizeof(glm::vec2));
        auto it = weld.find(key);
        if (it != weld.end()) {
            mesh.Indices.push_back(it->second);
            continue;
        }
        const uint32_t index = (uint32_t)mesh.Vertices.size();
        weld.emplace(std::move(key), index);
        mesh.Vertices.push_back(v);
        mesh.Indices.push_back(index);
    }
    std::vector<glm::vec3> tan(mesh.Vertices.size(), glm::vec3(0.0f)), bit(mesh.Vertices.size(), glm::vec3(0.0f));
    for (size_t t = 0; t + 2 < mesh.Indices.size(); t += 3) {
        const Vertex& a = mesh.Vertices[mesh.Indices[t]];
        const Vertex& b = mesh.Vertices[mesh.Indices[t + 1]];
        const Vertex& c = mesh.Vertices[mesh.Indices[t + 2]];
        const glm::vec3 e1 = b.Position - a.Position, e2 = c.Position - a.Position;
        const float s1 = b.TexCoord.x - a.TexCoord.x, t1 = b.TexCoord.y - a.TexCoord.y;
        const float s2 = c.TexCoord.x - a.TexCoord.x, t2 = c.TexCoord.y - a.TexCoord.y;
        const float det = s1 * t2 - s2 * t1;
        if (std::fabs(det) < 1e-20f) continue;
        const float r = 1.0f / det;
        const glm::vec3 T = (e1 * t2 - e2 * t1) * r, B = (e2 * s1 - e1 * s2) * r;
        for (int k = 0; k < 3; ++k) {
            tan[mesh.Indices[t + k]] = tan[mesh.Indices[t + k]] + T;
            bit[mesh.Indices[t + k]] = bit[mesh.Indices[t + k]] + B;
        }
    }
    for (size_t i = 0; i < mesh.Vertices.size(); ++i) {
        Vertex& v = mesh.Vertices[i];
        const glm::vec3 n = v.Normal;
        glm::vec3 T = tan[i] - n * glm::dot(n, tan[i]);  // Gram-Schmidt against the normal
        const float lt = glm::length(T), lb = glm::length(bit[i]);
        v.Tangent = lt > 0.0f ? T * (1.0f / lt) : glm::vec3(0.0f);
        v.Bitangent = lb > 0.0f ? bit[i] * (1.0f / lb) : glm::vec3(0.0f);
    }
    return mesh;
}

// ---- Wavefront OBJ / MTL -----------------------------------------------------------------------
struct ObjMaterial {
    glm::vec3 kd{0.6f, 0.6f, 0.6f};  // Assimp's ObjFile::Material default diffuse
    bool hasPm = false, hasPr = false;
    float pm = 1.0f, pr = 1.0f;
    std::string mapKd;
};

void ParseMtl(const fs::path& file, std::map<std::string, ObjMaterial>& out) {
    std::ifstream f(file);
    if (!f) {
        LogError("material library not found", file.string());
        return;
    }
    std::string line;
    ObjMaterial* cur = nullptr;
    while (std::getline(f, line)) {
        std::istringstream ls(line);
        std::string tok;
        if (!(ls >> tok) || tok[0] == '#') continue;
        if (tok == "newmtl") {
            std::string name;
            std::getline(ls >> std::ws, name);
            cur = &out[name];
            *cur = ObjMaterial{};
        } else if (!cur) {
            continue;
        } else if (tok == "Kd") {
            ls >> cur->kd.x >> cur->kd.y >> cur->kd.z;
        } else if (tok == "Pm") {
            cur->hasPm = static_cast<bool>(ls >> cur->pm);
        } else if (tok == "Pr") {
            cur->hasPr = static_cast<bool>(ls >> cur->pr);
        } else if (tok == "map_Kd") {
            std::string rest;
            std::getline(ls >> std::ws, rest);
            // options (-bm 1 ...) precede the file name: keep the last token
            const size_t sp = rest.find_last_of(" \t");
            cur->mapKd = sp == std::string::npos ? rest : rest.substr(sp + 1);
            while (!cur->mapKd.empty() && (cur->mapKd.back() == '\r' || cur->mapKd.back() == ' '))
                cur->mapKd.pop_back();
        }
    }
}

ModelData LoadObj(const fs::path& path) {
    ModelData data;
    std::ifstream f(path);
    if (!f) {
        LogError("model file not found", path.string());
        return data;
    }
    const fs::path dir = path.parent_path();
    std::vector<glm::vec3> pos, col, nrm;
    std::vector<glm::vec2> uvs;
    std::vector<bool> hasCol;
    std::map<std::string, ObjMaterial> mtl;
    std::unordered_map<std::string, int> materialIndex, texLookup;

    struct Group {
        std::vector<Corner> corners;
        bool allNormals = true;
        int material = -1;
    };
    std::vector<Group> groups;
    Group cur;
    std::string curMaterial;
    auto materialFor = [&](const std::string& name) -> int {
        auto it = materialIndex.find(name);
        if (it != materialIndex.end()) return it->second;
        const ObjMaterial m = mtl.count(name) ? mtl[name] : ObjMaterial{};
        Geometry::Material out{};
        out.BaseColorFactor = glm::vec4(m.kd, 1.0f);  // COLOR_DIFFUSE read into aiColor4D: alpha 1
        out.MetallicFactor = m.hasPm ? m.pm : 1.0f;   // ModelLoader.cpp:375-378 defaults
        out.RoughnessFactor = m.hasPr ? m.pr : 1.0f;
        out.BaseColorTextureIndex = ResolveTextureIndex(m.mapKd, dir, data, texLookup);
        const int index = (int)data.m_Materials.size();
        data.m_Materials.push_back(out);
        materialIndex.emplace(name, index);
        return index;
    };
    auto flush = [&]() {
        if (!cur.corners.empty()) {
            cur.material = materialFor(curMaterial);
            groups.push_back(std::move(cur));
        }
        cur = Group{};
    };
    auto resolve = [](long i, size_t n) -> long { return i > 0 ? i - 1 : (long)n + i; };

    std::string line;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ls(line);
        std::string tok;
        if (!(ls >> tok) || tok[0] == '#') continue;
        if (tok == "v") {
            glm::vec3 p{}, c{1.0f, 1.0f, 1.0f};
            ls >> p.x >> p.y >> p.z;
            float extra[3];
            bool color = static_cast<bool>(ls >> extra[0] >> extra[1] >> extra[2]);
            if (color) c = glm::vec3(extra[0], extra[1], extra[2]);
            pos.push_back(p);
            col.push_back(c);
            hasCol.push_back(color);
        } else if (tok == "vt") {
            glm::vec2 t{};
            ls >> t.x >> t.y;
            uvs.push_back(t);
        } else if (tok == "vn") {
            glm::vec3 n{};
            ls >> n.x >> n.y >> n.z;
            nrm.push_back(n);
        } else if (tok == "f") {
            std::vector<Corner> poly;
            bool polyNormals = true;
            std::string vtx;
            while (ls >> vtx) {
                long vi = 0, ti = 0, ni = 0;
                const size_t s1 = vtx.find('/');
                vi = std::strtol(vtx.c_str(), nullptr, 10);
                if (s1 != std::string::npos) {
                    const size_t s2 = vtx.find('/', s1 + 1);
                    if (s2 != s1 + 1) ti = std::strtol(vtx.c_str() + s1 + 1, nullptr, 10);
                    if (s2 != std::string::npos) ni = std::strtol(vtx.c_str() + s2 + 1, nullptr, 10);
                }
                const long v = resolve(vi, pos.size());
                if (v < 0 || (size_t)v >= pos.size()) {
                    LogError("face references a missing vertex", path.string());
                    return ModelData{};
                }
                Corner c{};
                c.p = pos[v];
                c.c = col[v];
                if (ti) {
                    const long t = resolve(ti, uvs.size());
                    if (t >= 0 && (size_t)t < uvs.size()) c.uv = uvs[t];
                }
                c.hasNormal = false;
                if (ni) {
                    const long n = resolve(ni, nrm.size());
                    if (n >= 0 && (size_t)n < nrm.size()) {
                        c.n = nrm[n];
                        c.hasNormal = true;
                    }
                }
                polyNormals = polyNormals && c.hasNormal;
                poly.push_back(c);
            }
            for (size_t k = 1; k + 1 < poly.size(); ++k) {  // aiProcess_Triangulate: fan from corner 0
                cur.corners.push_back(poly[0]);
                cur.corners.push_back(poly[k]);
                cur.corners.push_back(poly[k + 1]);
            }
            if (poly.size() >= 3) cur.allNormals = cur.allNormals && polyNormals;
        } else if (tok == "usemtl") {
            flush();
            std::getline(ls >> std::ws, curMaterial);
        } else if (tok == "o" || tok == "g") {
            flush();
        } else if (tok == "mtllib") {
            std::string lib;
            std::getline(ls >> std::ws, lib);
            ParseMtl(dir / lib, mtl);
        }
    }
    flush();
    for (Group& g : groups) {
        data.m_Meshes.push_back(BuildMesh(g.corners, g.allNormals, g.material));
    }
    if (data.m_Meshes.empty()) LogError("no triangles in", path.string());
    return data;
}

// ---- minimal JSON (glTF) -----------------------------------------------------------------------
struct Json {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    double num = 0.0;
    bool b = false;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json* get(const char* k) const {
        for (const auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    double numOr(const char* k, double d) const {
        const Json* j = get(k);
        return j && j->type == Number ? j->num : d;
    }
};

struct JsonParser {
    const char* p;
    const char* end;
    bool ok = true;
    void ws() {
        while (p < end && std::isspace((unsigned char)*p)) ++p;
    }
    Json parse() {
        ws();
        Json j;
        if (p >= end) { ok = false; return j; }
        const char c = *p;
        if (c == '{') {
            j.type = Json::Object;
            ++p;
            ws();
            if (p < end && *p == '}') { ++p; return j; }
            while (ok) {
                ws();
                Json k = parse();
                if (k.type != Json::String) { ok = false; break; }
                ws();
                if (p >= end || *p != ':') { ok = false; break; }
                ++p;
                j.obj.emplace_back(k.str, parse());
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == '}') { ++p; break; }
                ok = false;
            }
        } else if (c == '[') {
            j.type = Json::Array;
            ++p;
            ws();
            if (p < end && *p == ']') { ++p; return j; }
            while (ok) {
                j.arr.push_back(parse());
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == ']') { ++p; break; }
                ok = false;
            }
        } else if (c == '"') {
            j.type = Json::String;
            ++p;
            while (p < end && *p != '"') {
                if (*p == '\\' && p + 1 < end) {
                    ++p;
                    switch (*p) {
                        case 'n': j.str += '\n'; break;
                        case 't': j.str += '\t'; break;
                        case 'u': j.str += '?'; p += 4; break;  // names only; not needed exactly
                        default: j.str += *p;
                    }
                    ++p;
                } else {
                    j.str += *p++;
                }
            }
            if (p >= end) ok = false; else ++p;
        } else if (c == 't' || c == 'f') {
            j.type = Json::Bool;
            j.b = c == 't';
            p += j.b ? 4 : 5;
        } else if (c == 'n') {
            p += 4;
        } else {
            char* e = nullptr;
            j.type = Json::Number;
            j.num = std::strtod(p, &e);
            if (e == p) ok = false;
            p = e;
        }
        return j;
    }
};

bool Base64Decode(const std::string& in, std::string& out) {
    auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z') return c - 'A';
        if (c >= 'a' && c <= 'z') return c - 'a' + 26;
        if (c >= '0' && c <= '9') return c - '0' + 52;
        if (c == '+') return 62;
        if (c == '/') return 63;
        return -1;
    };
    out.clear();
    int buf = 0, bits = 0;
    for (char c : in) {
        if (c == '=') break;
        const int v = val(c);
        if (v < 0) continue;
        buf = (buf << 6) | v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back((char)((buf >> bits) & 0xFF));
        }
    }
    return true;
}

// glTF node transform: matrix, or T * R * S from translation / rotation (x, y, z, w) / scale.
glm::mat4 NodeMatrix(const Json& node) {
    glm::mat4 m(1.0f);
    if (const Json* mj = node.get("matrix"); mj && mj->arr.size() == 16) {
        for (int i = 0; i < 16; ++i) m[i / 4][i % 4] = (float)mj->arr[i].num;
        return m;
    }
    glm::vec3 t(0.0f), s(1.0f);
    glm::quat q(1.0f, 0.0f, 0.0f, 0.0f);
    if (const Json* tj = node.get("translation"); tj && tj->arr.size() == 3)
        t = glm::vec3((float)tj->arr[0].num, (float)tj->arr[1].num, (float)tj->arr[2].num);
    if (const Json* rj = node.get("rotation"); rj && rj->arr.size() == 4)
        q = glm::quat((float)rj->arr[3].num, (float)rj->arr[0].num, (float)rj->arr[1].num, (float)rj->arr[2].num);
    if (const Json* sj = node.get("scale"); sj && sj->arr.size() == 3)
        s = glm::vec3((float)sj->arr[0].num, (float)sj->arr[1].num, (float)sj->arr[2].num);
    return glm::scale(glm::translate(glm::mat4(1.0f), t) * glm::mat4_cast(q), s);
}

ModelData LoadGltf(const fs::path& path) {
    ModelData data;
    std::string file;
    if (!ReadFile(path.string(), file)) {
        LogError("model file not found", path.string());
        return data;
    }
    std::string jsonText, glbBin;
    if (file.size() >= 12 && std::memcmp(file.data(), "glTF", 4) == 0) {  // GLB container
        size_t off = 12;
        while (off + 8 <= file.size()) {
            uint32_t len, type;
            std::memcpy(&len, file.data() + off, 4);
            std::memcpy(&type, file.data() + off + 4, 4);
            if (off + 8 + len > file.size()) break;
            if (type == 0x4E4F534Au) jsonText.assign(file.data() + off + 8, len);
            else if (type == 0x004E4942u) glbBin.assign(file.data() + off + 8, len);
            off += 8 + ((len + 3) & ~3u);
        }
    } else {
        jsonText = file;
    }
    JsonParser jp{jsonText.data(), jsonText.data() + jsonText.size()};
    const Json root = jp.parse();
    if (!jp.ok || root.type != Json::Object) {
        LogError("malformed glTF JSON", path.string());
        return data;
    }
    const fs::path dir = path.parent_path();
    static const Json kEmpty;
    auto arrOf = [&](const char* k) -> const std::vector<Json>& {
        const Json* j = root.get(k);
        return j ? j->arr : kEmpty.arr;
    };
    std::vector<std::string> buffers;
    for (const Json& b : arrOf("buffers")) {
        std::string bytes;
        const Json* uri = b.get("uri");
        if (!uri) {
            bytes = glbBin;
        } else if (uri->str.rfind("data:", 0) == 0) {
            const size_t comma = uri->str.find(',');
            Base64Decode(comma == std::string::npos ? std::string() : uri->str.substr(comma + 1), bytes);
        } else if (!ReadFile((dir / uri->str).string(), bytes)) {
            LogError("glTF buffer not found", (dir / uri->str).string());
            return ModelData{};
        }
        buffers.push_back(std::move(bytes));
    }
    const std::vector<Json>& views = arrOf("bufferViews");
    const std::vector<Json>& accessors = arrOf("accessors");
    // accessor -> float components (normalised integer formats are converted) or indices
    auto readAccessor = [&](int index, int comps, std::vector<float>& out) -> bool {
        if (index < 0 || (size_t)index >= accessors.size()) return false;
        const Json& a = accessors[index];
        const size_t count = (size_t)a.numOr("count", 0);
        const int ctype = (int)a.numOr("componentType", 5126);
        const bool norm = a.get("normalized") && a.get("normalized")->b;
        out.assign(count * comps, 0.0f);
        const Json* bvj = a.get("bufferView");
        if (!bvj) return true;  // all zeros (sparse accessors are not supported)
        const int bvi = (int)bvj->num;
        if (bvi < 0 || (size_t)bvi >= views.size()) return false;
        const Json& bv = views[bvi];
        const int bi = (int)bv.numOr("buffer", 0);
        if (bi < 0 || (size_t)bi >= buffers.size()) return false;
        const std::string& buf = buffers[bi];
        const size_t csize = ctype == 5126 || ctype == 5125 ? 4 : (ctype == 5123 || ctype == 5122 ? 2 : 1);
        const size_t stride = bv.get("byteStride") ? (size_t)bv.numOr("byteStride", 0) : csize * comps;
        const size_t base = (size_t)bv.numOr("byteOffset", 0) + (size_t)a.numOr("byteOffset", 0);
        for (size_t i = 0; i < count; ++i)
            for (int c = 0; c < comps; ++c) {
                const size_t o = base + i * stride + c * csize;
                if (o + csize > buf.size()) return false;
                const unsigned char* q = reinterpret_cast<const unsigned char*>(buf.data() + o);
                float v = 0.0f;
                switch (ctype) {
                    case 5126: std::memcpy(&v, q, 4); break;
                    case 5125: { uint32_t u; std::memcpy(&u, q, 4); v = (float)u; break; }
                    case 5123: { uint16_t u; std::memcpy(&u, q, 2); v = norm ? u / 65535.0f : (float)u; break; }
                    case 5122: { int16_t s; std::memcpy(&s, q, 2); v = norm ? std::fmax(s / 32767.0f, -1.0f) : (float)s; break; }
                    case 5121: v = norm ? q[0] / 255.0f : (float)q[0]; break;
                    case 5120: { const int8_t s = (int8_t)q[0]; v = norm ? std::fmax(s / 127.0f, -1.0f) : (float)s; break; }
                    default: return false;
                }
                out[i * comps + c] = v;
            }
        return true;
    };
    // materials (pbrMetallicRoughness; glTF's own defaults are 1 / 1 / 1, like ModelLoader.cpp:375)
    const std::vector<Json>& images = arrOf("images");
    const std::vector<Json>& textures = arrOf("textures");
    std::unordered_map<std::string, int> texLookup;
    for (const Json& m : arrOf("materials")) {
        Geometry::Material out{};
        if (const Json* pbr = m.get("pbrMetallicRoughness")) {
            if (const Json* bc = pbr->get("baseColorFactor"); bc && bc->arr.size() == 4)
                out.BaseColorFactor = glm::vec4((float)bc->arr[0].num, (float)bc->arr[1].num, (float)bc->arr[2].num,
                                                (float)bc->arr[3].num);
            out.MetallicFactor = (float)pbr->numOr("metallicFactor", 1.0);
            out.RoughnessFactor = (float)pbr->numOr("roughnessFactor", 1.0);
            if (const Json* bt = pbr->get("baseColorTexture")) {
                const int ti = (int)bt->numOr("index", -1);
                if (ti >= 0 && (size_t)ti < textures.size()) {
                    const int ii = (int)textures[ti].numOr("source", -1);
                    if (ii >= 0 && (size_t)ii < images.size()) {
                        const Json* uri = images[ii].get("uri");
                        if (uri && uri->str.rfind("data:", 0) != 0)
                            out.BaseColorTextureIndex = ResolveTextureIndex(uri->str, dir, data, texLookup);
                        else
                            LogError("embedded textures are not supported", path.string());
                    }
                }
            }
        }
        data.m_Materials.push_back(out);
    }
    // meshes: one Geometry::Mesh per triangle primitive (Assimp splits primitives into meshes)
    std::vector<std::vector<size_t>> meshPrims;
    for (const Json& m : arrOf("meshes")) {
        std::vector<size_t> ids;
        const Json* prims = m.get("primitives");
        for (const Json& pr : prims ? prims->arr : kEmpty.arr) {
            if ((int)pr.numOr("mode", 4) != 4) continue;  // SortByPType: triangles only reach the renderer
            const Json* attrs = pr.get("attributes");
            if (!attrs || !attrs->get("POSITION")) continue;
            std::vector<float> P, N, T, C, I;
            if (!readAccessor((int)attrs->get("POSITION")->num, 3, P)) {
                LogError("bad POSITION accessor", path.string());
                return ModelData{};
            }
            const size_t nv = P.size() / 3;
            const bool hasN = attrs->get("NORMAL") && readAccessor((int)attrs->get("NORMAL")->num, 3, N);
            const bool hasT = attrs->get("TEXCOORD_0") && readAccessor((int)attrs->get("TEXCOORD_0")->num, 2, T);
            int ccomps = 0;
            if (const Json* cj = attrs->get("COLOR_0")) {
                const int ai = (int)cj->num;
                ccomps = (ai >= 0 && (size_t)ai < accessors.size() && accessors[ai].get("type") &&
                          accessors[ai].get("type")->str == "VEC4") ? 4 : 3;
                if (!readAccessor(ai, ccomps, C)) ccomps = 0;
            }
            if (const Json* ij = pr.get("indices")) {
                if (!readAccessor((int)ij->num, 1, I)) {
                    LogError("bad index accessor", path.string());
                    return ModelData{};
                }
            } else {
                I.resize(nv);
                for (size_t i = 0; i < nv; ++i) I[i] = (float)i;
            }
            std::vector<Corner> corners;
            corners.reserve(I.size());
            for (size_t k = 0; k + 2 < I.size(); k += 3)
                for (int e = 0; e < 3; ++e) {
                    const size_t v = (size_t)I[k + e];
                    if (v >= nv) {
                        LogError("index out of range", path.string());
                        return ModelData{};
                    }
                    Corner c{};
                    c.p = glm::vec3(P[3 * v], P[3 * v + 1], P[3 * v + 2]);
                    if (hasN) c.n = glm::vec3(N[3 * v], N[3 * v + 1], N[3 * v + 2]);
                    if (hasT) c.uv = glm::vec2(T[2 * v], T[2 * v + 1]);
                    c.c = ccomps ? glm::vec3(C[ccomps * v], C[ccomps * v + 1], C[ccomps * v + 2]) : glm::vec3(1.0f);
                    c.hasNormal = hasN;
                    corners.push_back(c);
                }
            const int mat = (int)pr.numOr("material", -1);
            ids.push_back(data.m_Meshes.size());
            data.m_Meshes.push_back(BuildMesh(corners, hasN, mat >= 0 && (size_t)mat < data.m_Materials.size() ? mat : -1));
        }
        meshPrims.push_back(std::move(ids));
    }
    // scene graph -> MeshInstance (parent * local, ModelLoader.cpp:505-540)
    const std::vector<Json>& nodes = arrOf("nodes");
    std::function<void(int, const glm::mat4&, int)> visit = [&](int n, const glm::mat4& parent, int depth) {
        if (n < 0 || (size_t)n >= nodes.size() || depth > 64) return;
        const Json& node = nodes[n];
        const glm::mat4 model = parent * NodeMatrix(node);
        const int mi = (int)node.numOr("mesh", -1);
        if (mi >= 0 && (size_t)mi < meshPrims.size())
            for (size_t id : meshPrims[mi]) {
                MeshInstance inst;
                inst.m_MeshIndex = id;
                inst.m_ModelMatrix = model;
                inst.m_NodeName = node.get("name") ? node.get("name")->str : std::string();
                data.m_MeshInstances.push_back(inst);
            }
        if (const Json* ch = node.get("children"))
            for (const Json& c : ch->arr) visit((int)c.num, model, depth + 1);
    };
    const std::vector<Json>& scenes = arrOf("scenes");
    const int sceneIndex = (int)root.numOr("scene", 0);
    if (sceneIndex >= 0 && (size_t)sceneIndex < scenes.size()) {
        if (const Json* sn = scenes[sceneIndex].get("nodes"))
            for (const Json& n : sn->arr) visit((int)n.num, glm::mat4(1.0f), 0);
    }
    return data;
}

bool ReadPnmToken(const std::string& s, size_t& i, std::string& tok) {
    tok.clear();
    while (i < s.size()) {
        if (s[i] == '#') {
            while (i < s.size() && s[i] != '\n') ++i;
        } else if (std::isspace((unsigned char)s[i])) {
            ++i;
        } else {
            break;
        }
    }
    while (i < s.size() && !std::isspace((unsigned char)s[i])) tok += s[i++];
    return !tok.empty();
}

}  // namespace

ModelData ModelLoader::Load(const std::string& filePath) {
    if (filePath.empty()) {
        LogError("empty file path", "");
        return {};
    }
    const std::string n = NormalizePath(filePath);
    if (!fs::exists(n)) {
        LogError("model file not found", n);
        return {};
    }
    const std::string ext = Lower(fs::path(n).extension().string());
    if (ext == ".obj") return LoadObj(n);
    if (ext == ".gltf" || ext == ".glb") return LoadGltf(n);
    LogError("unsupported model format (Assimp is not linked)", n);
    return {};
}

namespace {
// One image file -> top-to-bottom RGBA8 rows (PNG, JPEG or PPM/PAM), unflipped. Width 0 on failure.
TextureData DecodeImageFile(const std::string& filePath) {
    TextureData t;
    std::string s;
    if (!ReadFile(NormalizePath(filePath), s)) {
        LogError("texture file not found", filePath);
        return t;
    }
    if (IsPng(s)) {
        std::string err;
        if (!DecodePng(s, t.Width, t.Height, t.Pixels, err)) {
            LogError(("PNG decode failed: " + err).c_str(), filePath);
            return TextureData{};
        }
        t.Channels = 4;
        return t;
    }
    if (IsJpeg(s)) {
        std::string err;
        if (!DecodeJpeg(s, t.Width, t.Height, t.Pixels, err)) {
            LogError(("JPEG decode failed: " + err).c_str(), filePath);
            return TextureData{};
        }
        t.Channels = 4;
        return t;
    }
    size_t i = 0;
    std::string magic, tok;
    if (!ReadPnmToken(s, i, magic)) return t;
    int w = 0, h = 0, maxv = 0, depth = 0;
    if (magic == "P6") {
        int* fields[3] = {&w, &h, &maxv};
        for (int* f : fields) {
            if (!ReadPnmToken(s, i, tok)) return t;
            *f = std::atoi(tok.c_str());
        }
        depth = 3;
    } else if (magic == "P7") {
        while (ReadPnmToken(s, i, tok) && tok != "ENDHDR") {
            std::string v;
            if (tok == "TUPLTYPE") { ReadPnmToken(s, i, v); continue; }
            if (!ReadPnmToken(s, i, v)) return t;
            if (tok == "WIDTH") w = std::atoi(v.c_str());
            else if (tok == "HEIGHT") h = std::atoi(v.c_str());
            else if (tok == "DEPTH") depth = std::atoi(v.c_str());
            else if (tok == "MAXVAL") maxv = std::atoi(v.c_str());
        }
    } else {
        LogError("unsupported image format (stb_image is not linked)", filePath);
        return t;
    }
    ++i;  // the single whitespace byte after the header
    if (w <= 0 || h <= 0 || maxv != 255 || (depth != 3 && depth != 4) || i + (size_t)w * h * depth > s.size()) {
        LogError("unsupported or truncated image", filePath);
        return t;
    }
    t.Width = w;
    t.Height = h;
    t.Channels = 4;
    t.Pixels.resize((size_t)w * h * 4);
    for (int y = 0; y < h; ++y) {
        const unsigned char* src = reinterpret_cast<const unsigned char*>(s.data() + i) + (size_t)y * w * depth;
        uint8_t* dst = t.Pixels.data() + (size_t)y * w * 4;
        for (int x = 0; x < w; ++x) {
            dst[4 * x + 0] = src[depth * x + 0];
            dst[4 * x + 1] = src[depth * x + 1];
            dst[4 * x + 2] = src[depth * x + 2];
            dst[4 * x + 3] = depth == 4 ? src[depth * x + 3] : 255;
        }
    }
    return t;
}
}  // namespace

TextureData TextureLoader::Load(const std::string& filePath) {
    TextureData t = DecodeImageFile(filePath);
    if (t.Width > 0) FlipRowsVertically(t.Pixels, t.Width, t.Height);  // stbi_set_flip_vertically_on_load(true)
    return t;
}

CubemapTextureData SkyboxTextureLoader::LoadFromFaces(const std::array<std::string, 6>& faces) {
    static const char* names[6] = {"+X", "-X", "+Y", "-Y", "+Z", "-Z"};
    CubemapTextureData out;
    for (int f = 0; f < 6; ++f) {
        if (faces[f].empty()) {
            LogError("cubemap face has an empty path", names[f]);
            return {};
        }
        const std::string ext = Lower(fs::path(faces[f]).extension().string());
        if (ext == ".exr") {
            LogError("EXR cubemap faces need tinyexr (not linked)", faces[f]);
            return {};
        }
        const TextureData t = DecodeImageFile(faces[f]);  // stbi_set_flip_vertically_on_load(false)
        if (t.Width <= 0) return {};
        if (f == 0) {
            out.m_Width = (uint32_t)t.Width;
            out.m_Height = (uint32_t)t.Height;
        } else if ((uint32_t)t.Width != out.m_Width || (uint32_t)t.Height != out.m_Height) {
            LogError("cubemap faces must share the same resolution", faces[f]);
            return {};
        }
        out.m_PixelData.insert(out.m_PixelData.end(), t.Pixels.begin(), t.Pixels.end());
    }
    out.m_MipCount = 1;
    return out;
}

namespace {
const char* const kFaceTokens[6][2] = {{"posx", "px"}, {"negx", "nx"}, {"posy", "py"},
                                       {"negy", "ny"}, {"posz", "pz"}, {"negz", "nz"}};

std::vector<fs::path> SortedFiles(const fs::path& dir) {
    std::vector<fs::path> files;
    std::error_code ec;
    for (const auto& e : fs::directory_iterator(dir, ec))
        if (e.is_regular_file()) files.push_back(e.path());
    std::sort(files.begin(), files.end());
    return files;
}
}  // namespace

CubemapTextureData SkyboxTextureLoader::LoadFromDirectory(const std::string& dir) {
    std::error_code ec;
    if (!fs::is_directory(dir, ec)) {
        LogError("cubemap directory is invalid", dir);
        return {};
    }
    std::array<std::vector<std::string>, 6> candidates;
    for (const fs::path& p : SortedFiles(dir)) {
        const std::string stem = Lower(p.stem().string());
        for (int f = 0; f < 6; ++f) {  // TryMatchFaceIndex: the first face whose token matches
            if (stem.find(kFaceTokens[f][0]) != std::string::npos || stem.find(kFaceTokens[f][1]) != std::string::npos) {
                candidates[f].push_back(p.string());
                break;
            }
        }
    }
    std::array<std::string, 6> faces;
    for (int f = 0; f < 6; ++f) {
        if (candidates[f].empty()) {
            LogError("missing cubemap face in directory", dir);
            return {};
        }
        faces[f] = candidates[f].front();  // no EXR candidates are usable here, so the first match
    }
    return LoadFromFaces(faces);
}

CubemapTextureData DiscoverDefaultSkybox(const std::string& assetsDir, std::string& source) {
    source.clear();
    const fs::path root = fs::path(assetsDir) / "Skyboxes";
    std::error_code ec;
    if (fs::exists(root / "DefaultSkybox.ktx", ec)) {  // Renderer.cpp:3831-3837
        LogError("KTX cubemaps are not restated; DefaultSkybox.ktx loads as invalid", (root / "DefaultSkybox.ktx").string());
        source = "DefaultSkybox.ktx";
        return {};
    }
    if (fs::exists(root / "Default", ec)) {  // :3840-3845
        source = "Default directory";
        return SkyboxTextureLoader::LoadFromDirectory((root / "Default").string());
    }
    if (!fs::is_directory(root, ec)) return {};
    std::array<std::string, 6> faces;  // :3848-3915: loose faces, short or long tokens
    std::array<bool, 6> found{};
    for (const fs::path& p : SortedFiles(root)) {
        const std::string stem = Lower(p.stem().string());
        for (int f = 0; f < 6; ++f) {
            if (found[f]) continue;
            for (const char* tok : kFaceTokens[f]) {
                if (stem.find(tok) != std::string::npos) {
                    faces[f] = p.string();
                    found[f] = true;
                    break;
                }
            }
        }
    }
    if (!std::all_of(found.begin(), found.end(), [](bool b) { return b; })) {
        LogError("PNG fallback skybox faces are incomplete", root.string());
        return {};
    }
    CubemapTextureData d = SkyboxTextureLoader::LoadFromFaces(faces);
    if (d.IsValid()) source = "PNG fallback";
    return d;
}

// glm::decompose (gtx/matrix_decompose.inl) without perspective / skew use, then
// glm::eulerAngles (pitch, yaw, roll) in degrees.
bool DecomposeMatrixToTransform(const glm::mat4& m, Transform& out) {
    out = Transform{};
    if (m[3][3] == 0.0f) return false;
    glm::mat4 local = m;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) local[i][j] /= m[3][3];
    glm::vec3 row[3];
    for (int i = 0; i < 3; ++i) row[i] = glm::vec3(local[i][0], local[i][1], local[i][2]);
    glm::vec3 scale;
    scale.x = glm::length(row[0]);
    if (scale.x == 0.0f) return false;
    row[0] = row[0] * (1.0f / scale.x);
    float skewXY = glm::dot(row[0], row[1]);
    row[1] = row[1] + row[0] * -skewXY;
    scale.y = glm::length(row[1]);
    if (scale.y == 0.0f) return false;
    row[1] = row[1] * (1.0f / scale.y);
    float skewXZ = glm::dot(row[0], row[2]);
    row[2] = row[2] + row[0] * -skewXZ;
    float skewYZ = glm::dot(row[1], row[2]);
    row[2] = row[2] + row[1] * -skewYZ;
    scale.z = glm::length(row[2]);
    if (scale.z == 0.0f) return false;
    row[2] = row[2] * (1.0f / scale.z);
    if (glm::dot(row[0], glm::cross(row[1], row[2])) < 0.0f) {
        for (int i = 0; i < 3; ++i) {
            scale[i] *= -1.0f;
            row[i] = row[i] * -1.0f;
        }
    }
    glm::quat q;
    const float trace = row[0].x + row[1].y + row[2].z;
    if (trace > 0.0f) {
        float root = std::sqrt(trace + 1.0f);
        q.w = 0.5f * root;
        root = 0.5f / root;
        q.x = root * (row[1].z - row[2].y);
        q.y = root * (row[2].x - row[0].z);
        q.z = root * (row[0].y - row[1].x);
    } else {
        static const int next[3] = {1, 2, 0};
        int i = 0;
        if (row[1].y > row[0].x) i = 1;
        if (row[2].z > row[i][i]) i = 2;
        const int j = next[i], k = next[j];
        float root = std::sqrt(row[i][i] - row[j][j] - row[k][k] + 1.0f);
        float qv[3];
        qv[i] = 0.5f * root;
        root = 0.5f / root;
        qv[j] = root * (row[i][j] + row[j][i]);
        qv[k] = root * (row[i][k] + row[k][i]);
        q.w = root * (row[j][k] - row[k][j]);
        q.x = qv[0]; q.y = qv[1]; q.z = qv[2];
    }
    q = glm::normalize(q);
    // glm::eulerAngles: pitch (x), yaw (y), roll (z)
    const float yr = 2.0f * (q.y * q.z + q.w * q.x);
    const float xr = q.w * q.w - q.x * q.x - q.y * q.y + q.z * q.z;
    const float pitch = (yr == 0.0f && xr == 0.0f) ? 2.0f * std::atan2(q.x, q.w) : std::atan2(yr, xr);
    const float yaw = std::asin(glm::clamp(-2.0f * (q.x * q.z - q.w * q.y), -1.0f, 1.0f));
    const float roll = std::atan2(2.0f * (q.x * q.y + q.w * q.z), q.w * q.w + q.x * q.x - q.y * q.y - q.z * q.z);
    const float toDeg = 57.295779513082320876798154814105f;
    out.Position = glm::vec3(local[3][0], local[3][1], local[3][2]);
    out.Scale = scale;
    out.Rotation = glm::vec3(pitch * toDeg, yaw * toDeg, roll * toDeg);
    return true;
}

}  // namespace Loader
}  // namespace Trident

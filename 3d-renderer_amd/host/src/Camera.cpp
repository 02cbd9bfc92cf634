// Camera.cpp — EditorCamera (EditorCamera.cpp:1-161) and RuntimeCamera (RuntimeCamera.cpp:1-203)
// matrix conventions.
#include "trident/Camera.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace Trident {

namespace {
constexpr float s_MinimumOrthographicSize = 0.01f;
constexpr float s_MinimumFieldOfView = 1.0f;
constexpr float s_MaximumFieldOfView = 179.0f;
constexpr float s_MinimumClipDistance = 0.001f;
bool eq(float a, float b) { return std::fabs(a - b) <= std::numeric_limits<float>::epsilon(); }
}  // namespace

EditorCamera::EditorCamera() {
    RecalculateOrientation();
    RecalculateProjectionMatrix();
    RecalculateViewMatrix();
}

void EditorCamera::SetPosition(const glm::vec3& position) {
    m_Position = position;
    RecalculateViewMatrix();
}

void EditorCamera::SetRotation(const glm::vec3& eulerDegrees) {
    m_Rotation = eulerDegrees;
    RecalculateOrientation();
    RecalculateViewMatrix();
}

void EditorCamera::SetProjectionType(ProjectionType type) {
    if (m_ProjectionType == type) return;
    m_ProjectionType = type;
    RecalculateProjectionMatrix();
}

void EditorCamera::SetFieldOfView(float fov) {
    const float c = glm::clamp(fov, s_MinimumFieldOfView, s_MaximumFieldOfView);
    if (eq(m_FieldOfView, c)) return;
    m_FieldOfView = c;
    RecalculateProjectionMatrix();
}

void EditorCamera::SetOrthographicSize(float size) {
    const float c = std::max(size, s_MinimumOrthographicSize);
    if (eq(m_OrthographicSize, c)) return;
    m_OrthographicSize = c;
    RecalculateProjectionMatrix();
}

void EditorCamera::SetClipPlanes(float nearClip, float farClip) {
    const float n = std::max(nearClip, s_MinimumClipDistance);
    const float f = std::max(farClip, n + s_MinimumClipDistance);
    if (eq(m_NearClip, n) && eq(m_FarClip, f)) return;
    m_NearClip = n;
    m_FarClip = f;
    RecalculateProjectionMatrix();
}

void EditorCamera::SetViewportSize(const glm::vec2& viewportSize) {
    glm::vec2 s = viewportSize;
    if (s.x <= 0.0f) s.x = 1.0f;
    if (s.y <= 0.0f) s.y = 1.0f;
    if (eq(m_ViewportSize.x, s.x) && eq(m_ViewportSize.y, s.y)) return;
    m_ViewportSize = s;
    RecalculateProjectionMatrix();
}

void EditorCamera::Invalidate() {
    RecalculateOrientation();
    RecalculateProjectionMatrix();
    RecalculateViewMatrix();
}

glm::vec3 EditorCamera::GetForwardDirection() const { return glm::rotate(m_Orientation, glm::vec3(0.0f, 0.0f, -1.0f)); }
glm::vec3 EditorCamera::GetRightDirection() const { return glm::rotate(m_Orientation, glm::vec3(1.0f, 0.0f, 0.0f)); }
glm::vec3 EditorCamera::GetUpDirection() const { return glm::rotate(m_Orientation, glm::vec3(0.0f, 1.0f, 0.0f)); }

void EditorCamera::RecalculateOrientation() { m_Orientation = glm::quat(glm::radians(m_Rotation)); }

void EditorCamera::RecalculateViewMatrix() {  // inverse(R * T) = mat4_cast(conj(q)) * translate(-p)
    const glm::mat4 rotation = glm::mat4_cast(glm::conjugate(m_Orientation));
    const glm::mat4 translation = glm::translate(glm::mat4(1.0f), -m_Position);
    m_ViewMatrix = rotation * translation;
}

void EditorCamera::RecalculateProjectionMatrix() {
    const float aspect = std::max(m_ViewportSize.x / std::max(m_ViewportSize.y, 0.0001f), 0.0001f);
    if (m_ProjectionType == ProjectionType::Orthographic) {
        const float hh = m_OrthographicSize * 0.5f, hw = hh * aspect;
        m_ProjectionMatrix = glm::orthoRH_ZO(-hw, hw, -hh, hh, m_NearClip, m_FarClip);
    } else {
        m_ProjectionMatrix = glm::perspectiveRH_ZO(glm::radians(m_FieldOfView), aspect, m_NearClip, m_FarClip);
    }
    m_ProjectionMatrix[1][1] *= -1.0f;  // Vulkan Y flip (EditorCamera.cpp:159)
}

// ---- RuntimeCamera ------------------------------------------------------------------------------
const glm::mat4& RuntimeCamera::GetViewMatrix() const {
    if (m_ViewDirty) {  // RuntimeCamera::UpdateViewMatrix (RuntimeCamera.cpp:166-175)
        const glm::quat q = BuildOrientation();
        const glm::vec3 fwd = q * glm::vec3(0.0f, 0.0f, -1.0f);
        const glm::vec3 up = q * glm::vec3(0.0f, 1.0f, 0.0f);
        m_ViewMatrix = glm::lookAt(m_Position, m_Position + fwd, up);
        m_ViewDirty = false;
    }
    return m_ViewMatrix;
}

const glm::mat4& RuntimeCamera::GetProjectionMatrix() const {
    if (m_ProjectionDirty) {  // RuntimeCamera::UpdateProjectionMatrix (RuntimeCamera.cpp:177-195)
        const float aspect = (m_ViewportSize.y > 0.0f) ? (m_ViewportSize.x / m_ViewportSize.y) : 1.0f;
        if (m_ProjectionType == ProjectionType::Perspective) {
            m_ProjectionMatrix = glm::perspective(glm::radians(m_FieldOfView), aspect, m_NearClip, m_FarClip);
            m_ProjectionMatrix[1][1] *= -1.0f;
        } else {
            const float oh = m_OrthographicSize, ow = oh * aspect;
            m_ProjectionMatrix = glm::ortho(-ow, ow, -oh, oh, m_NearClip, m_FarClip);
        }
        m_ProjectionDirty = false;
    }
    return m_ProjectionMatrix;
}

void RuntimeCamera::SetPosition(const glm::vec3& p) {
    if (p == m_Position) return;
    m_Position = p;
    m_ViewDirty = true;
}
void RuntimeCamera::SetRotation(const glm::vec3& r) {
    if (r == m_Rotation) return;
    m_Rotation = r;
    m_ViewDirty = true;
}
void RuntimeCamera::SetProjectionType(ProjectionType type) {
    if (type == m_ProjectionType) return;
    m_ProjectionType = type;
    m_ProjectionDirty = true;
}
void RuntimeCamera::SetFieldOfView(float fov) {
    if (eq(m_FieldOfView, fov)) return;
    m_FieldOfView = fov;
    m_ProjectionDirty = true;
}
void RuntimeCamera::SetOrthographicSize(float size) {
    if (eq(m_OrthographicSize, size)) return;
    m_OrthographicSize = size;
    m_ProjectionDirty = true;
}
void RuntimeCamera::SetClipPlanes(float n, float f) {
    if (eq(m_NearClip, n) && eq(m_FarClip, f)) return;
    m_NearClip = n;
    m_FarClip = f;
    m_ProjectionDirty = true;
}
void RuntimeCamera::SetViewportSize(const glm::vec2& s) {
    if (std::fabs(m_ViewportSize.x - s.x) <= 0.0001f && std::fabs(m_ViewportSize.y - s.y) <= 0.0001f) return;
    m_ViewportSize = s;
    m_ProjectionDirty = true;
}
glm::vec3 RuntimeCamera::GetForwardDirection() const { return BuildOrientation() * glm::vec3(0.0f, 0.0f, -1.0f); }
glm::quat RuntimeCamera::BuildOrientation() const { return glm::normalize(glm::quat(glm::radians(m_Rotation))); }

}  // namespace Trident

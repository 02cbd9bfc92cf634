// Camera.h — Trident's camera contract (Renderer/Camera/Camera.h) and the two implementations the
// renderer routes between: EditorCamera (perspectiveRH_ZO + Vulkan Y flip, EditorCamera.cpp:126-160)
// and RuntimeCamera (glm::perspective = RH_NO + Y flip, lookAt view; RuntimeCamera.cpp:166-203).
#pragma once

#include "glm_subset.h"

namespace Trident {

class Camera {
public:
    enum class ProjectionType { Perspective = 0, Orthographic };
    virtual ~Camera() = default;
    virtual const glm::mat4& GetViewMatrix() const = 0;
    virtual const glm::mat4& GetProjectionMatrix() const = 0;
    virtual glm::vec3 GetPosition() const = 0;
    virtual glm::vec3 GetRotation() const = 0;
    virtual void SetPosition(const glm::vec3& position) = 0;
    virtual void SetRotation(const glm::vec3& eulerDegrees) = 0;
    virtual void SetProjectionType(ProjectionType type) = 0;
    virtual ProjectionType GetProjectionType() const = 0;
    virtual void SetFieldOfView(float fieldOfViewDegrees) = 0;
    virtual float GetFieldOfView() const = 0;
    virtual void SetOrthographicSize(float size) = 0;
    virtual float GetOrthographicSize() const = 0;
    virtual void SetClipPlanes(float nearClip, float farClip) = 0;
    virtual float GetNearClip() const = 0;
    virtual float GetFarClip() const = 0;
    virtual void SetViewportSize(const glm::vec2& viewportSize) = 0;
    virtual glm::vec2 GetViewportSize() const = 0;
    virtual void Invalidate() = 0;
};

class EditorCamera : public Camera {
public:
    EditorCamera();
    const glm::mat4& GetViewMatrix() const override { return m_ViewMatrix; }
    const glm::mat4& GetProjectionMatrix() const override { return m_ProjectionMatrix; }
    glm::vec3 GetPosition() const override { return m_Position; }
    glm::vec3 GetRotation() const override { return m_Rotation; }
    void SetPosition(const glm::vec3& position) override;
    void SetRotation(const glm::vec3& eulerDegrees) override;
    void SetProjectionType(ProjectionType type) override;
    ProjectionType GetProjectionType() const override { return m_ProjectionType; }
    void SetFieldOfView(float fieldOfViewDegrees) override;
    float GetFieldOfView() const override { return m_FieldOfView; }
    void SetOrthographicSize(float size) override;
    float GetOrthographicSize() const override { return m_OrthographicSize; }
    void SetClipPlanes(float nearClip, float farClip) override;
    float GetNearClip() const override { return m_NearClip; }
    float GetFarClip() const override { return m_FarClip; }
    void SetViewportSize(const glm::vec2& viewportSize) override;
    glm::vec2 GetViewportSize() const override { return m_ViewportSize; }
    void Invalidate() override;
    glm::vec3 GetForwardDirection() const;
    glm::vec3 GetRightDirection() const;
    glm::vec3 GetUpDirection() const;

private:
    void RecalculateOrientation();
    void RecalculateViewMatrix();
    void RecalculateProjectionMatrix();
    glm::vec3 m_Position{0.0f, 0.0f, 5.0f};
    glm::vec3 m_Rotation{0.0f};
    glm::quat m_Orientation{1.0f, 0.0f, 0.0f, 0.0f};
    glm::vec2 m_ViewportSize{1280.0f, 720.0f};
    float m_FieldOfView{60.0f};
    float m_OrthographicSize{20.0f};
    float m_NearClip{0.1f};
    float m_FarClip{1000.0f};
    ProjectionType m_ProjectionType{ProjectionType::Perspective};
    glm::mat4 m_ViewMatrix{1.0f};
    glm::mat4 m_ProjectionMatrix{1.0f};
};

class RuntimeCamera : public Camera {
public:
    RuntimeCamera() = default;
    const glm::mat4& GetViewMatrix() const override;
    const glm::mat4& GetProjectionMatrix() const override;
    glm::vec3 GetPosition() const override { return m_Position; }
    glm::vec3 GetRotation() const override { return m_Rotation; }
    void SetPosition(const glm::vec3& position) override;
    void SetRotation(const glm::vec3& eulerDegrees) override;
    void SetProjectionType(ProjectionType type) override;
    ProjectionType GetProjectionType() const override { return m_ProjectionType; }
    void SetFieldOfView(float fieldOfViewDegrees) override;
    float GetFieldOfView() const override { return m_FieldOfView; }
    void SetOrthographicSize(float size) override;
    float GetOrthographicSize() const override { return m_OrthographicSize; }
    void SetClipPlanes(float nearClip, float farClip) override;
    float GetNearClip() const override { return m_NearClip; }
    float GetFarClip() const override { return m_FarClip; }
    void SetViewportSize(const glm::vec2& viewportSize) override;
    glm::vec2 GetViewportSize() const override { return m_ViewportSize; }
    void Invalidate() override { m_ViewDirty = m_ProjectionDirty = true; }
    glm::vec3 GetForwardDirection() const;

private:
    glm::quat BuildOrientation() const;
    glm::vec3 m_Position{0.0f, 1.8f, 6.0f};
    glm::vec3 m_Rotation{0.0f};
    glm::vec2 m_ViewportSize{1280.0f, 720.0f};
    float m_FieldOfView{60.0f};
    float m_OrthographicSize{20.0f};
    float m_NearClip{0.1f};
    float m_FarClip{1000.0f};
    ProjectionType m_ProjectionType{ProjectionType::Perspective};
    mutable glm::mat4 m_ViewMatrix{1.0f};
    mutable glm::mat4 m_ProjectionMatrix{1.0f};
    mutable bool m_ViewDirty{true};
    mutable bool m_ProjectionDirty{true};
};

}  // namespace Trident

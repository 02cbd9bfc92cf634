// RenderCommand.cpp — the process-wide renderer behind the static facade (Startup::GetRenderer()).
#include "trident/RenderCommand.h"

namespace Trident {

Renderer& RenderCommand::GetRenderer() {
    static Renderer s_Renderer;
    return s_Renderer;
}

}  // namespace Trident

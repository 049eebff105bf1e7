// Captured-graph introspection: the kernel nodes of a hipGraph by name (diagnostics and tests -- e.g. that a
// tensor-parallel decode graph holds no collective-library kernel). torch.cuda.CUDAGraph(keep_graph=True)
// exposes the graph handle (raw_cuda_graph()).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <vector>

extern "C" {

// Newline-separated names of the graph's kernel nodes (capture order of hipGraphGetNodes) into buf (NUL-terminated,
// truncated at cap bytes); other node kinds appear as "<type N>". Returns the node count, or -1 on an API error.
int nls_graph_kernel_names(void* graph, char* buf, long cap) {
  size_t n = 0;
  if (hipGraphGetNodes((hipGraph_t)graph, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes((hipGraph_t)graph, nodes.data(), &n) != hipSuccess) return -1;
  long used = 0;
  if (cap > 0) buf[0] = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) return -1;
    char line[512];
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams p;
      if (hipGraphKernelNodeGetParams(nodes[i], &p) != hipSuccess) return -1;
      const char* name = hipKernelNameRefByPtr(p.func, nullptr);
      snprintf(line, sizeof(line), "%s\n", name ? name : "<unnamed kernel>");
    } else {
      snprintf(line, sizeof(line), "<type %d>\n", (int)t);
    }
    const long l = (long)strlen(line);
    if (used + l + 1 <= cap) {
      memcpy(buf + used, line, (size_t)l + 1);
      used += l;
    }
  }
  return (int)n;
}

}  // extern "C"

/* The Python interpreter as an executable of our own, linked with a sanitizer runtime (tools/sanitize_host.sh):
 * extension modules built with -fsanitize=address,undefined or -fsanitize=thread (upow_amd._build --variant)
 * resolve the runtime from this executable when they are imported, so the pybind11 modules' Python tests
 * run instrumented without preloading anything. */
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }

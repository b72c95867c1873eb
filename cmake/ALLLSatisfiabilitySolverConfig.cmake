# CMake package of the MI355X ALLL solver, consumable exactly like the reference's package
# (example/CMakeLists.txt:67,73):
#     find_package(ALLLSatisfiabilitySolver CONFIG REQUIRED)
#     target_link_libraries(app ALLLSatisfiabilitySolver)
# with -DALLLSatisfiabilitySolver_DIR=<repo>/cmake.  The target carries the compatibility
# headers (SATInstance.h, Clause.h, VariablesArray.h, RandomBoolGenerator.h) and links the
# C-ABI library liballl.so (HIP kernels for gfx950) plus OpenMP (main.cpp calls
# omp_get_num_procs through SATInstance.h, as with the reference).
get_filename_component(_ALLL_ROOT "${CMAKE_CURRENT_LIST_DIR}/.." ABSOLUTE)
include(CMakeFindDependencyMacro)
find_dependency(OpenMP REQUIRED)
if(NOT TARGET ALLLSatisfiabilitySolver)
    set(_ALLL_LIB "${_ALLL_ROOT}/alllsatisfiabilitysolver_amd/liballl.so")
    if(NOT EXISTS "${_ALLL_LIB}")
        message(FATAL_ERROR "ALLLSatisfiabilitySolver: ${_ALLL_LIB} not built (run make in ${_ALLL_ROOT})")
    endif()
    add_library(ALLLSatisfiabilitySolver::alll SHARED IMPORTED)
    set_target_properties(ALLLSatisfiabilitySolver::alll PROPERTIES IMPORTED_LOCATION "${_ALLL_LIB}")
    add_library(ALLLSatisfiabilitySolver INTERFACE IMPORTED)
    set_target_properties(ALLLSatisfiabilitySolver PROPERTIES
        INTERFACE_INCLUDE_DIRECTORIES "${_ALLL_ROOT}/include/alll_compat;${_ALLL_ROOT}/include"
        INTERFACE_LINK_LIBRARIES "ALLLSatisfiabilitySolver::alll;OpenMP::OpenMP_CXX")
endif()
set(ALLLSatisfiabilitySolver_FOUND TRUE)

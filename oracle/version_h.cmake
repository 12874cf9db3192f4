# oracle/version_h.cmake -- TEST INFRASTRUCTURE ONLY (oracle/Makefile target `progs`).
# The reference's programs include <version.h>, which its CMakeLists.txt:42 generates from
# src/version.h.in with configure_file().  This script runs that same configure_file() on the
# reference's own template, with the version taken from the reference's project() line
# (CMakeLists.txt:3), and writes the header under oracle/_ref/gen/.  Nothing is hand-written.
#   cmake -DREF=/root/reference -DOUT=oracle/_ref/gen/version.h -P oracle/version_h.cmake
file(STRINGS "${REF}/CMakeLists.txt" _proj REGEX "^project\\(.*VERSION [0-9]+\\.[0-9]+\\.[0-9]+")
string(REGEX MATCH "VERSION ([0-9]+)\\.([0-9]+)\\.([0-9]+)" _v "${_proj}")
set(CMAKE_PROJECT_VERSION_MAJOR ${CMAKE_MATCH_1})
set(CMAKE_PROJECT_VERSION_MINOR ${CMAKE_MATCH_2})
set(CMAKE_PROJECT_VERSION_PATCH ${CMAKE_MATCH_3})
set(CMAKE_PROJECT_VERSION "${CMAKE_MATCH_1}.${CMAKE_MATCH_2}.${CMAKE_MATCH_3}")
configure_file("${REF}/src/version.h.in" "${OUT}")

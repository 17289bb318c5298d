"""Built native artefacts (libnm03.so, _nm03*.so) land here; see build.py / CMakeLists.txt."""

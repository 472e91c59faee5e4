// `conv` executable: see app.hpp / cli.hpp.
#include "pconv/app.hpp"

int main(int argc, char** argv) { return pconv::conv_main(argc, argv); }

// Prints the reference's galois.cpp constant tables (GINV, GEXP, GMULT) as JSON hex
// strings.  Links the reference source in place; used only to produce the committed
// fixture tests/golden/galois_tables.json (tests/golden/make_galois_fixture.py).
#include <cstdio>
#include "galois.h"

static void hex(const char* name, const unsigned char* p, int n, bool last)
{
    std::printf("  \"%s\": \"", name);
    for (int i = 0; i < n; ++i) std::printf("%02x", p[i]);
    std::printf("\"%s\n", last ? "" : ",");
}

int main()
{
    std::printf("{\n");
    hex("GINV", Norm::GINV, 256, false);
    hex("GEXP", Norm::GEXP, 512, false);
    hex("GMULT", &Norm::GMULT[0][0], 65536, true);
    std::printf("}\n");
    return 0;
}

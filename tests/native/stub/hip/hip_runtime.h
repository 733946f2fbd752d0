// empty stand-in: host builds of the restated libm headers (tests/native)
#pragma once

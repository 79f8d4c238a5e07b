// the adapter's own header, at the path the reference tree gives it (include/backend/)
#include "../../../adapter/hipOptimizer.h"

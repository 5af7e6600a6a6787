"""Where libfc2.so is (no imports beyond os: the prestart loads it before numpy is imported)."""
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfc2.so")
# A/B measurements only (scripts/ab_build.sh): load another in-tree build of the library instead
if os.environ.get("FC2_LIB_VARIANT"):
    LIB_PATH = os.path.join(_HERE, "libfc2_%s.so" % os.environ["FC2_LIB_VARIANT"])

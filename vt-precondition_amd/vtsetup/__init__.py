"""vtsetup: entry layer of the Krylov path (config in vtconfig/, step object with main())."""
from .config import DEFAULT_XML, Etree, SolverConfig  # noqa: F401

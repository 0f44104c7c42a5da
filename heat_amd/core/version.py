"""Version of the framework (API level of the reference it matches: Heat 1.1.1 + pending additions)."""
major: int = 0
minor: int = 1
micro: int = 0
extension: str = "mi355x"
__version__: str = "{}.{}.{}-{}".format(major, minor, micro, extension)
reference_api: str = "heat 1.1.1"

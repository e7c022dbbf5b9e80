import AsyncTools.AsyncPPO  # noqa: F401
import AsyncTools.utils  # noqa: F401
import AsyncTools.envs  # noqa: F401

from vstyler.flow_match import FlowMatchScheduler  # noqa: F401
